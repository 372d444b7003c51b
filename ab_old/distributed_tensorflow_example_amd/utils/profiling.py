"""Tracing / profiling: the reference only prints wall-clock
AvgTime over 100-step windows (example.py:143-183).  Here:

* `StepTimer`   -- per-step GPU intervals from hipEvents (falls back to wall
                   clock on CPU); p50 / p90 / mean, the BASELINE step-time metric;
* `range(name)` -- a roctx range (visible in `rocprofv3 --marker-trace`) and,
                   when a `TraceRecorder` is active, a Chrome-trace event;
* `TraceRecorder` -- host ranges to chrome://tracing / Perfetto JSON.

    with profiling.TraceRecorder("trace.json"):
        with profiling.range("fwd"): ...
"""
from __future__ import annotations

import contextlib
import json
import os
import statistics
import threading
import time
from typing import List, Optional

import torch

_tls = threading.local()
_recorder: Optional["TraceRecorder"] = None


def _roctx():
    try:
        from .. import _native

        return _native.load()
    except Exception:  # noqa: BLE001 - profiling must never break training
        return None


class TraceRecorder:
    def __init__(self, path: str, pid: Optional[int] = None):
        self.path = path
        self.pid = pid if pid is not None else int(os.environ.get("RANK", 0))
        self.events: List[dict] = []
        self.t0 = time.perf_counter()
        self._lock = threading.Lock()

    def add(self, name: str, start: float, end: float, cat: str = "host", args: Optional[dict] = None):
        ev = {"name": name, "ph": "X", "cat": cat, "pid": self.pid, "tid": threading.get_ident() % 100000,
              "ts": (start - self.t0) * 1e6, "dur": (end - start) * 1e6}
        if args:
            ev["args"] = args
        with self._lock:
            self.events.append(ev)

    def save(self):
        d = os.path.dirname(os.path.abspath(self.path))
        os.makedirs(d, exist_ok=True)
        with open(self.path, "w") as f:
            json.dump({"traceEvents": self.events, "displayTimeUnit": "ms"}, f)

    def __enter__(self):
        global _recorder
        self._prev = _recorder
        _recorder = self
        return self

    def __exit__(self, *exc):
        global _recorder
        _recorder = self._prev
        self.save()
        return False


@contextlib.contextmanager
def range(name: str, sync: bool = False):  # noqa: A001 - mirrors roctx naming
    """roctx range + optional Chrome-trace event; `sync` waits for the GPU at
    both ends so the host interval covers the device work."""
    C = _roctx()
    if sync and torch.cuda.is_available():
        torch.cuda.synchronize()
    t = time.perf_counter()
    if C is not None:
        C.roctx_push(name)
    try:
        yield
    finally:
        if sync and torch.cuda.is_available():
            torch.cuda.synchronize()
        if C is not None:
            C.roctx_pop()
        if _recorder is not None:
            _recorder.add(name, t, time.perf_counter())


def mark(name: str):
    C = _roctx()
    if C is not None:
        C.roctx_mark(name)


class StepTimer:
    """Per-step durations: hipEvent pairs on GPU, perf_counter on CPU."""

    def __init__(self, device=None):
        self.gpu = device is not None and torch.device(device).type == "cuda"
        self._open = None
        self.pending = []
        self.ms: List[float] = []

    def start(self):
        if self.gpu:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._open = e
        else:
            self._open = time.perf_counter()

    def stop(self, steps: int = 1):
        if self.gpu:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.pending.append((self._open, e, steps))
        else:
            self.ms.append((time.perf_counter() - self._open) * 1e3 / steps)
        self._open = None

    def _drain(self):
        if self.pending:
            torch.cuda.synchronize()
            for a, b, n in self.pending:
                self.ms.append(a.elapsed_time(b) / n)
            self.pending = []

    def summary(self) -> dict:
        self._drain()
        if not self.ms:
            return {"steps": 0}
        s = sorted(self.ms)
        q = lambda p: s[min(len(s) - 1, int(round(p * (len(s) - 1))))]  # noqa: E731
        return {"steps": len(s), "p50_ms": q(0.5), "p90_ms": q(0.9), "p99_ms": q(0.99),
                "mean_ms": statistics.fmean(s), "min_ms": s[0], "max_ms": s[-1]}
