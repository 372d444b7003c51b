"""TensorBoard summaries without TensorFlow.

Reference: `tf.scalar_summary("cost", cross_entropy)`, `tf.merge_all_summaries()`,
`tf.train.SummaryWriter(logs_path, graph)` and `writer.add_summary(summary, step)`
every step (example.py:130-135,154,171).  Summary ops are deferred Tensors
producing a serialized `Summary` proto; FileWriter appends TFRecord-framed
`Event` protos through the native asynchronous writer (masked CRC32C,
csrc/runtime/tfrecord.cpp), so per-step summaries never block the loop.
`summary_iterator` reads event files back (tests, tooling).
"""
from __future__ import annotations

import os
import socket
import struct
import time
from typing import Iterator, List, Optional

import numpy as np
import torch

from .. import _native
from .graph import SUMMARIES, Tensor, get_default_graph


# ----------------------------------------------------------------------- proto bits
def _varint(v: int) -> bytes:
    out = bytearray()
    v &= (1 << 64) - 1
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _key(field: int, wt: int) -> bytes:
    return _varint((field << 3) | wt)


def _len_field(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def scalar_value(tag: str, value: float) -> bytes:
    return _len_field(1, tag.encode()) + _key(2, 5) + struct.pack("<f", float(value))


def summary_proto(values: List[bytes]) -> bytes:
    return b"".join(_len_field(1, v) for v in values)


def histogram_value(tag: str, values, bins: int = 30) -> bytes:
    arr = np.asarray(values, dtype=np.float64).reshape(-1).tolist()
    return _native.load().encode_histogram_value(tag, arr, bins)


def _read_varint(b: bytes, i: int):
    shift = v = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << shift
        if not c & 0x80:
            return v, i
        shift += 7


def parse_fields(b: bytes):
    i, out = 0, []
    while i < len(b):
        k, i = _read_varint(b, i)
        f, wt = k >> 3, k & 7
        if wt == 0:
            v, i = _read_varint(b, i)
        elif wt == 1:
            v = b[i:i + 8]
            i += 8
        elif wt == 5:
            v = b[i:i + 4]
            i += 4
        elif wt == 2:
            n, i = _read_varint(b, i)
            v = b[i:i + n]
            i += n
        else:
            raise ValueError("bad wire type")
        out.append((f, wt, v))
    return out


class Event:
    def __init__(self, raw: bytes):
        self.wall_time = 0.0
        self.step = 0
        self.file_version = None
        self.graph_def = None
        self.summary = []  # list of (tag, simple_value or None, kind)
        for f, wt, v in parse_fields(raw):
            if f == 1 and wt == 1:
                self.wall_time = struct.unpack("<d", v)[0]
            elif f == 2 and wt == 0:
                self.step = v
            elif f == 3:
                self.file_version = v.decode()
            elif f == 4:
                self.graph_def = v
            elif f == 5:
                for f2, _, val in parse_fields(v):
                    if f2 != 1:
                        continue
                    tag, sv, kind = None, None, "unknown"
                    for f3, wt3, x in parse_fields(val):
                        if f3 == 1:
                            tag = x.decode()
                        elif f3 == 2 and wt3 == 5:
                            sv, kind = struct.unpack("<f", x)[0], "scalar"
                        elif f3 == 5:
                            kind = "histo"
                    self.summary.append((tag, sv, kind))


    def scalars(self):
        return [(t, v) for t, v, k in self.summary if k == "scalar"]


def summary_iterator(path: str) -> Iterator[Event]:
    for rec in _native.load().read_records(path, True):
        yield Event(rec)


# ----------------------------------------------------------------------- ops
def _to_float(x):
    if isinstance(x, torch.Tensor):
        # a scalar is read as is (no reduction kernel on the device)
        return float(x.item()) if x.numel() == 1 else float(x.detach().float().mean().item())
    return float(np.asarray(x, dtype=np.float64).mean())


def scalar(name: str, tensor, collections=None, family=None) -> Tensor:
    t = Tensor(lambda v: summary_proto([scalar_value(name, _to_float(v))]), [tensor], "ScalarSummary")
    for c in (collections or [SUMMARIES]):
        get_default_graph().add_to_collection(c, t)
    return t


def histogram(name: str, values, collections=None, family=None) -> Tensor:
    def f(v):
        arr = v.detach().float().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)
        return summary_proto([histogram_value(name, arr)])
    t = Tensor(f, [values], "HistogramSummary")
    for c in (collections or [SUMMARIES]):
        get_default_graph().add_to_collection(c, t)
    return t


def merge(inputs, collections=None, name=None) -> Tensor:
    return Tensor(lambda *vs: b"".join(v for v in vs if v), list(inputs), name or "MergeSummary")


def merge_all(key=SUMMARIES) -> Optional[Tensor]:
    s = get_default_graph().get_collection(key)
    return merge(s) if s else None


# TF 0.x names used by the reference
scalar_summary = scalar
histogram_summary = histogram
merge_summary = merge
merge_all_summaries = merge_all


# ----------------------------------------------------------------------- writer
class FileWriter:
    """tf.summary.FileWriter / tf.train.SummaryWriter."""

    def __init__(self, logdir: str, graph=None, max_queue: int = 4096, flush_secs: float = 2.0,
                 filename_suffix: str = ""):
        os.makedirs(logdir, exist_ok=True)
        fn = f"events.out.tfevents.{int(time.time()):010d}.{socket.gethostname()}.{os.getpid()}{filename_suffix}"
        self.path = os.path.join(logdir, fn)
        self._w = _native.load().EventFileWriter(self.path, flush_secs, max_queue)
        self.logdir = logdir
        if graph is not None:
            self.add_graph(graph)

    def add_summary(self, summary, global_step=None):
        if summary is None:
            return
        if isinstance(summary, (np.ndarray, np.generic)):
            summary = summary.item() if summary.ndim == 0 else bytes(summary)
        step = int(global_step) if global_step is not None else 0
        self._w.add_summary(bytes(summary), step)

    def add_scalar(self, tag: str, value: float, global_step: int = 0, wall_time: float = 0.0):
        self._w.add_scalar(tag, float(value), int(global_step), wall_time)

    def add_scalars(self, values: dict, global_step: int = 0):
        self.add_summary(summary_proto([scalar_value(k, v) for k, v in values.items()]), global_step)

    def add_histogram(self, tag: str, values, global_step: int = 0):
        self.add_summary(summary_proto([histogram_value(tag, values)]), global_step)

    def add_graph(self, graph, global_step=None):
        gd = graph.as_graph_def() if hasattr(graph, "as_graph_def") else bytes(graph)
        self._w.add_graph(gd)

    def add_event(self, event: bytes):
        self._w.add_event(event)

    def flush(self):
        self._w.flush()

    def close(self):
        self._w.close()

    def get_logdir(self):
        return self.logdir

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


SummaryWriter = FileWriter


class FileWriterCache:
    _cache = {}

    @classmethod
    def get(cls, logdir):
        if logdir not in cls._cache:
            cls._cache[logdir] = FileWriter(logdir)
        return cls._cache[logdir]

    @classmethod
    def clear(cls):
        for w in cls._cache.values():
            w.close()
        cls._cache.clear()
