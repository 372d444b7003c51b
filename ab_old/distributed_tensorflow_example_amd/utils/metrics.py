"""JSON-lines metrics sink: one record per event, rank-tagged,
line-buffered, safe to tail while a job runs.  Complements the tfevents
writer (TensorBoard) and the console step line."""
from __future__ import annotations

import json
import os
import threading
import time
from typing import Optional


class MetricsWriter:
    def __init__(self, path: str, rank: Optional[int] = None, also_stdout: bool = False):
        self.path = path
        self.rank = rank if rank is not None else int(os.environ.get("RANK", 0))
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        self._f = open(path, "a", buffering=1)
        self._lock = threading.Lock()
        self.also_stdout = also_stdout

    def write(self, kind: str, step: Optional[int] = None, **values):
        rec = {"t": round(time.time(), 6), "rank": self.rank, "kind": kind}
        if step is not None:
            rec["step"] = int(step)
        for k, v in values.items():
            rec[k] = float(v) if hasattr(v, "__float__") and not isinstance(v, (int, bool, str)) else v
        line = json.dumps(rec)
        with self._lock:
            self._f.write(line + "\n")
        if self.also_stdout:
            print(line, flush=True)

    def close(self):
        with self._lock:
            self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False


def read_jsonl(path: str):
    with open(path) as f:
        return [json.loads(l) for l in f if l.strip()]
