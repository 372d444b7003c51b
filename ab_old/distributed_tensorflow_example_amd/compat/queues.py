"""Queue-based input pipelines: FIFOQueue, QueueRunner, Coordinator, batch.

Reference: lr2.py:158-175 (FIFOQueue(capacity) + enqueue_many/dequeue +
tf.train.batch, closed with cancel_pending_enqueues), input_pipeline.py
(slice_input_producer + read_file + decode_jpeg + batch, Coordinator +
start_queue_runners) and input_pipeline_large_dataset.py (feeder thread,
enqueue_many, RunOptions(timeout_in_ms)).  Queue storage is the native
bounded blocking queue (csrc/runtime/blocking_queue.cpp); every wait happens
with the GIL released so feeder threads really run concurrently.
"""
from __future__ import annotations

import threading
import time
from typing import Any, List, Optional, Sequence

import numpy as np
import torch

from .. import _native
from .graph import (QUEUE_RUNNERS, Operation, RunContext, Tensor, _to_tensor, get_default_graph)


class OutOfRangeError(Exception):
    """Queue closed and exhausted (tf.errors.OutOfRangeError)."""


class DeadlineExceededError(Exception):
    """Operation timed out (tf.errors.DeadlineExceededError)."""


class CancelledError(Exception):
    pass


def _timeout(ctx: Optional[RunContext]) -> float:
    opts = getattr(ctx, "options", None) if ctx is not None else None
    if opts is not None and getattr(opts, "timeout_in_ms", 0):
        return opts.timeout_in_ms / 1000.0
    return -1.0


def _host(v):
    if isinstance(v, torch.Tensor):
        return v.detach().cpu().numpy()
    return v


class FIFOQueue:
    def __init__(self, capacity: int, dtypes, shapes=None, names=None, shared_name=None, name="fifo_queue"):
        C = _native.load()
        self._q = C.BlockingQueue(int(capacity))
        self._C = C
        self.capacity = int(capacity)
        self.dtypes = list(dtypes) if isinstance(dtypes, (list, tuple)) else [dtypes]
        self.shapes = shapes
        self.names = names
        self.name = name

    # host-level API (used by feeder threads and QueueRunners)
    def put(self, item, timeout: float = -1.0):
        try:
            self._q.put(item, timeout)
        except self._C.QueueClosedError:
            raise CancelledError("Enqueue operation was cancelled (queue closed)")
        except self._C.QueueTimeoutError:
            raise DeadlineExceededError("enqueue timed out")

    def get(self, timeout: float = -1.0):
        try:
            return self._q.get(timeout)
        except self._C.QueueClosedError:
            raise OutOfRangeError(f"FIFOQueue '{self.name}' is closed and has insufficient elements")
        except self._C.QueueTimeoutError:
            raise DeadlineExceededError("dequeue timed out")

    def get_many(self, n: int, timeout: float = -1.0, allow_smaller=False):
        try:
            return self._q.get_many(int(n), timeout, allow_smaller)
        except self._C.QueueClosedError:
            raise OutOfRangeError(f"FIFOQueue '{self.name}' is closed and has insufficient elements")
        except self._C.QueueTimeoutError:
            raise DeadlineExceededError("dequeue_many timed out")

    # graph ops
    def enqueue(self, vals, name=None) -> Operation:
        vals = vals if isinstance(vals, (list, tuple)) else [vals]

        def f(*v):
            self.put(tuple(_host(x) for x in v))
        return Operation(f, list(vals), name or "enqueue")

    def enqueue_many(self, vals, name=None) -> Operation:
        vals = vals if isinstance(vals, (list, tuple)) else [vals]

        def f(*v):
            cols = [_host(x) for x in v]
            n = len(cols[0])
            for i in range(n):
                self.put(tuple(c[i] for c in cols))
        return Operation(f, list(vals), name or "enqueue_many")

    def _components(self, t: Tensor, name: str):
        # TF returns one tensor per component; they share the (memoised) dequeue
        if len(self.dtypes) <= 1:
            return t
        return [Tensor(lambda v, i=i: v[i], [t], f"{name}_{i}") for i in range(len(self.dtypes))]

    def dequeue(self, name=None):
        t = Tensor(None, [], name or "dequeue")
        q = self

        def ev(ctx):
            item = q.get(_timeout(ctx))
            return item[0] if len(item) == 1 else list(item)
        t._eval = ev
        return self._components(t, name or "dequeue")

    def dequeue_many(self, n, name=None):
        t = Tensor(None, [], name or "dequeue_many")
        q = self

        def ev(ctx):
            items = q.get_many(n, _timeout(ctx))
            return _stack_items(items)
        t._eval = ev
        return self._components(t, name or "dequeue_many")

    def dequeue_up_to(self, n, name=None):
        t = Tensor(None, [], name or "dequeue_up_to")
        q = self

        def ev(ctx):
            return _stack_items(q.get_many(n, _timeout(ctx), True))
        t._eval = ev
        return self._components(t, name or "dequeue_up_to")

    def close(self, cancel_pending_enqueues: bool = False, name=None) -> Operation:
        return Operation(lambda: self._q.close(cancel_pending_enqueues), [], name or "close")

    def size(self, name=None) -> Tensor:
        return Tensor(lambda: torch.tensor(self._q.size()), [], name or "size")

    def is_closed(self):
        return self._q.closed()


def _stack_items(items):
    if not items:
        return []
    ncol = len(items[0])
    cols = []
    for c in range(ncol):
        vals = [it[c] for it in items]
        if isinstance(vals[0], (bytes, str)):
            cols.append(np.array(vals, dtype=object))
        else:
            cols.append(np.stack([np.asarray(v) for v in vals]))
    return cols[0] if ncol == 1 else cols


class RandomShuffleQueue(FIFOQueue):
    """Shuffling variant: dequeue picks a random buffered element (min_after_dequeue kept)."""

    def __init__(self, capacity, min_after_dequeue, dtypes, shapes=None, seed=None, **kw):
        super().__init__(capacity, dtypes, shapes, **kw)
        self._buf: List[Any] = []
        self._min = int(min_after_dequeue)
        self._rng = np.random.default_rng(seed)
        self._lock = threading.Lock()

    def get(self, timeout: float = -1.0):
        while True:
            with self._lock:
                if len(self._buf) > self._min or (self.is_closed() and self._buf):
                    i = int(self._rng.integers(len(self._buf)))
                    self._buf[i], self._buf[-1] = self._buf[-1], self._buf[i]
                    return self._buf.pop()
            try:
                item = super().get(0.05 if timeout < 0 else timeout)
            except DeadlineExceededError:
                if timeout >= 0:
                    raise
                continue
            with self._lock:
                self._buf.append(item)


# ----------------------------------------------------------------------- runners
class Coordinator:
    def __init__(self, clean_stop_exception_types=None):
        self._stop = threading.Event()
        self._exc = None
        self._lock = threading.Lock()
        self._threads: List[threading.Thread] = []
        self._clean = tuple(clean_stop_exception_types or (OutOfRangeError,))

    def request_stop(self, ex=None):
        with self._lock:
            if ex is not None and self._exc is None and not isinstance(ex, self._clean):
                self._exc = ex
            self._stop.set()

    def should_stop(self) -> bool:
        return self._stop.is_set()

    def wait_for_stop(self, timeout=None) -> bool:
        return self._stop.wait(timeout)

    def clear_stop(self):
        self._stop.clear()
        self._exc = None

    def register_thread(self, t):
        self._threads.append(t)

    def stop_on_exception(self):
        coord = self

        class _CM:
            def __enter__(self):
                return coord

            def __exit__(self, et, ev, tb):
                if ev is not None:
                    coord.request_stop(ev)
                return True
        return _CM()

    def join(self, threads=None, stop_grace_period_secs=120, ignore_live_threads=False):
        threads = list(threads or []) + self._threads
        deadline = time.time() + stop_grace_period_secs
        for t in threads:
            t.join(max(0.0, deadline - time.time()) if self._stop.is_set() else None)
        live = [t for t in threads if t.is_alive()]
        if self._exc is not None:
            raise self._exc
        if live and not ignore_live_threads:
            raise RuntimeError(f"Coordinator stopped with threads still running: {[t.name for t in live]}")

    @property
    def joined(self):
        return all(not t.is_alive() for t in self._threads)


class QueueRunner:
    def __init__(self, queue: FIFOQueue = None, enqueue_ops=None, close_op=None, cancel_op=None,
                 queue_closed_exception_types=None):
        self.queue = queue
        self.enqueue_ops = list(enqueue_ops or [])
        self.close_op = close_op if close_op is not None else (queue.close() if queue else None)
        self.cancel_op = cancel_op if cancel_op is not None else (queue.close(True) if queue else None)
        self.exceptions_raised = []

    def _run(self, sess, op, coord):
        try:
            while coord is None or not coord.should_stop():
                sess.run(op)
        except (OutOfRangeError, CancelledError):
            try:
                if self.close_op is not None:
                    sess.run(self.close_op)
            except Exception:
                pass
        except Exception as e:  # surface real errors through the coordinator
            self.exceptions_raised.append(e)
            if coord is not None:
                coord.request_stop(e)
            else:
                raise

    def create_threads(self, sess, coord=None, daemon=True, start=False):
        threads = []
        for op in self.enqueue_ops:
            t = threading.Thread(target=self._run, args=(sess, op, coord), daemon=daemon,
                                 name=f"QueueRunner-{getattr(self.queue, 'name', 'q')}")
            threads.append(t)
        if coord is not None:
            closer = threading.Thread(target=self._close_on_stop, args=(sess, coord), daemon=True)
            threads.append(closer)
            for t in threads:
                coord.register_thread(t)
        if start:
            for t in threads:
                t.start()
        return threads

    def _close_on_stop(self, sess, coord):
        coord.wait_for_stop()
        try:
            if self.cancel_op is not None:
                sess.run(self.cancel_op)
        except Exception:
            pass


def add_queue_runner(qr, collection=QUEUE_RUNNERS):
    get_default_graph().add_to_collection(collection, qr)


def start_queue_runners(sess=None, coord=None, daemon=True, start=True, collection=QUEUE_RUNNERS):
    from .session import get_default_session

    sess = sess or get_default_session()
    threads = []
    for qr in get_default_graph().get_collection(collection):
        threads += qr.create_threads(sess, coord=coord, daemon=daemon, start=start)
    return threads


# ----------------------------------------------------------------------- producers / batching
def batch(tensors, batch_size, num_threads=1, capacity=32, enqueue_many=False, shapes=None,
          allow_smaller_final_batch=False, name="batch"):
    """Background threads evaluate `tensors` and enqueue; returns dequeue_many."""
    single = not isinstance(tensors, (list, tuple))
    tlist = [tensors] if single else list(tensors)
    q = FIFOQueue(max(capacity, batch_size), [None] * len(tlist), name=name + "/fifo_queue")
    enq = q.enqueue_many(tlist) if enqueue_many else q.enqueue(tlist)
    add_queue_runner(QueueRunner(q, [enq] * num_threads))
    out = q.dequeue_up_to(batch_size) if allow_smaller_final_batch else q.dequeue_many(batch_size)
    return out if single else list(out) if len(tlist) > 1 else [out]


def shuffle_batch(tensors, batch_size, capacity, min_after_dequeue, num_threads=1, seed=None,
                  enqueue_many=False, name="shuffle_batch"):
    tlist = tensors if isinstance(tensors, (list, tuple)) else [tensors]
    q = RandomShuffleQueue(capacity, min_after_dequeue, [None] * len(tlist), seed=seed, name=name)
    enq = q.enqueue_many(tlist) if enqueue_many else q.enqueue(tlist)
    add_queue_runner(QueueRunner(q, [enq] * num_threads))
    out = q.dequeue_many(batch_size)
    if not isinstance(tensors, (list, tuple)):
        return out
    return list(out) if len(tlist) > 1 else [out]


def slice_input_producer(tensor_list, num_epochs=None, shuffle=True, seed=None, capacity=32,
                         name="input_producer"):
    """One row of each input per dequeue, cycling epochs (input_pipeline.py:60-62)."""
    tl = list(tensor_list)
    q = FIFOQueue(capacity, [None] * len(tl), name=name)
    state = {"epoch": 0}
    rng = np.random.default_rng(seed)

    def feed(*vals):
        cols = [_host(v) if not isinstance(v, list) else v for v in vals]
        n = len(cols[0])
        if num_epochs is not None and state["epoch"] >= num_epochs:
            q._q.close(False)
            raise OutOfRangeError("epochs exhausted")
        order = rng.permutation(n) if shuffle else np.arange(n)
        state["epoch"] += 1
        for i in order:
            q.put(tuple(c[i] for c in cols))
    add_queue_runner(QueueRunner(q, [Operation(feed, tl, name + "/enqueue")]))
    deq = q.dequeue()
    return [deq] if len(tl) == 1 else list(deq)


def string_input_producer(string_tensor, num_epochs=None, shuffle=True, seed=None, capacity=32,
                          name="input_producer"):
    return slice_input_producer([string_tensor], num_epochs, shuffle, seed, capacity, name)[0]


def read_file(filename, name="ReadFile") -> Tensor:
    from ..utils.gfile import GFile

    def f(fn):
        fn = fn.decode() if isinstance(fn, bytes) else str(fn)
        with GFile(fn, "rb") as fh:
            return fh.read()
    return Tensor(f, [filename], name)


def decode_jpeg(contents, channels=0, name="DecodeJpeg") -> Tensor:
    def f(b):
        import io

        from PIL import Image

        img = Image.open(io.BytesIO(b))
        if channels == 1:
            img = img.convert("L")
        elif channels == 3:
            img = img.convert("RGB")
        arr = np.asarray(img, dtype=np.uint8)
        if arr.ndim == 2 and channels != 0:
            arr = arr[:, :, None]
        return torch.from_numpy(arr.copy())
    return Tensor(f, [contents], name)


decode_image = decode_jpeg
decode_png = decode_jpeg
