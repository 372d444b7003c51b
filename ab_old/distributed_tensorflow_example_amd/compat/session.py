"""Session: evaluates fetches of the deferred graph (compat/graph.py).

`Session(target).run(fetches, feed_dict)` follows TF-1 structure rules:
fetches may be a single Tensor/Variable/Operation, or nested lists / tuples /
dicts of them; Operations return None; values come back as numpy arrays
(python scalars for 0-d).  All fetches of one call share one RunContext, so
e.g. `[train_op, cross_entropy, summary_op, global_step]` (example.py:168-170)
runs the forward pass once.
"""
from __future__ import annotations

import contextlib
import threading
from typing import Any

import numpy as np
import torch

from . import lowering as _lowering
from . import resident as _resident
from .graph import Operation, RunContext, Tensor, get_default_graph

_tls = threading.local()


class ConfigProto:
    def __init__(self, allow_soft_placement=True, log_device_placement=False, **kw):
        self.allow_soft_placement = allow_soft_placement
        self.log_device_placement = log_device_placement
        self.__dict__.update(kw)


class RunOptions:
    FULL_TRACE = 3
    NO_TRACE = 0

    def __init__(self, timeout_in_ms: int = 0, trace_level: int = 0):
        self.timeout_in_ms = timeout_in_ms
        self.trace_level = trace_level


class RunMetadata:
    def __init__(self):
        self.step_stats = None


_SCALARS = (np.float32, np.float64, np.int64, np.int32)   # seeded fetch values, returned as they are


def _to_numpy(v):
    if v is None:
        return None
    if isinstance(v, torch.Tensor):
        a = v.detach()
        if a.dtype == torch.bfloat16:
            a = a.float()
        a = a.cpu().numpy()
        return a[()] if a.ndim == 0 else a
    if isinstance(v, (list, tuple)):
        return type(v)(_to_numpy(x) for x in v)
    return v


def _flat(fetches) -> list:
    if type(fetches) is list and all(isinstance(f, Tensor) for f in fetches):
        return fetches                      # the common shape: a flat list of graph nodes
    return _lowering._flatten(fetches, [])


class Session:
    def __init__(self, target: str = "", graph=None, config: ConfigProto = None):
        self.target = target
        self.graph = graph or get_default_graph()
        self.config = config
        self._closed = False
        self._ctx_stack = []
        self._post_run = []
        self._in_post = False
        self._lower = _lowering.enabled()   # DTF_GRAPH_LOWERING, read once per session (not per run)
        # {fetch ids: runner}: lowered plans' direct runners for a flat fetch list
        # (compat/lowering.py _PlanBase.fast_runner) -- feed dict in, outputs out,
        # None = not this run (then the full path runs)
        self._fast = {}

    # ---------------------------------------------------------------- run
    def run(self, fetches, feed_dict=None, options: RunOptions = None, run_metadata=None):
        if self._closed:
            raise RuntimeError("Attempted to use a closed Session.")
        if self._fast and type(fetches) is list and options is None and feed_dict is not None:
            fk = tuple(map(id, fetches))
            fast = self._fast.get(fk)
            if fast is not None:
                out = fast(feed_dict)
                if out is not None:
                    if self._post_run and not self._in_post:
                        self._post_hooks()
                    return out
        ctx = RunContext(feed_dict or {}, self.graph.device)
        ctx.session = self
        ctx.options = options
        flat = _flat(fetches)
        _lowering.try_lower(self, fetches, ctx, flat)   # fused steps for matched train ops
        if _resident._LIVE and not getattr(ctx, "resident_ran", False):
            _resident.quiesce_all()      # this run may write variables a resident engine holds
        for f in flat:                   # async train ops: pull the ps variables first
            hook = getattr(f, "_pre_run", None)
            if hook is not None:
                hook()
        if flat is fetches:              # flat list of graph nodes: no per-fetch dispatch
            memo, out = ctx.memo, []
            for f in fetches:
                v = memo[id(f)] if id(f) in memo else ctx.eval(f)
                out.append(None if f._is_op else (v if type(v) in _SCALARS else _to_numpy(v)))
        else:
            out = self._run(fetches, ctx)
        if self._post_run and not self._in_post:
            self._post_hooks()
        return out

    def _post_hooks(self):
        # step-boundary services (Supervisor checkpoints): run in the training
        # thread between steps, never concurrently with a train op
        self._in_post = True
        try:
            for cb in list(self._post_run):
                cb(self)
        finally:
            self._in_post = False

    def _run(self, f, ctx):
        if f is None:
            return None
        if isinstance(f, (list, tuple)):
            vals = [self._run(x, ctx) for x in f]
            return vals if isinstance(f, list) else tuple(vals)
        if isinstance(f, dict):
            return {k: self._run(v, ctx) for k, v in f.items()}
        if isinstance(f, str):                 # "y:0" / "train_op" fetch by name
            f = self.graph.get_tensor_by_name(f)
        if isinstance(f, Tensor):
            v = ctx.eval(f)
            return None if f._is_op else _to_numpy(v)
        if callable(f):
            return _to_numpy(f(ctx))
        raise TypeError(f"Fetch argument {f!r} has invalid type {type(f)}")

    def make_callable(self, fetches, feed_list=None):
        feed_list = list(feed_list or [])

        def call(*args):
            return self.run(fetches, feed_dict=dict(zip(feed_list, args)))
        return call

    # ---------------------------------------------------------------- lifecycle
    def close(self):
        _resident.quiesce_all()
        self._closed = True

    @property
    def closed(self):
        return self._closed

    def as_default(self):
        return _default_session(self)

    def __enter__(self):
        cm = _default_session(self)
        cm.__enter__()
        self._ctx_stack.append(cm)
        return self

    def __exit__(self, *exc):
        cm = self._ctx_stack.pop()
        cm.__exit__(*exc)
        self.close()
        return False


class InteractiveSession(Session):
    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        _stack().append(self)


def _stack():
    s = getattr(_tls, "stack", None)
    if s is None:
        s = _tls.stack = []
    return s


@contextlib.contextmanager
def _default_session(sess):
    _stack().append(sess)
    try:
        yield sess
    finally:
        _stack().pop()


def get_default_session():
    s = _stack()
    if not s:
        raise RuntimeError("No default session is registered. Use `with sess.as_default()` or pass session.")
    return s[-1]
