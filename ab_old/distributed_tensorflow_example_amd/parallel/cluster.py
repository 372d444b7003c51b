"""Cluster topology and rendezvous (ClusterSpec -> ranks, native TCP store).

Reference: `tf.train.ClusterSpec({"ps": [...], "worker": [...]})` built from
hard-coded host lists (example.py:23-30) or cluster_conf.json (lr2.py:325-327);
task index = position in the job's list.  Every task ran a TF gRPC server.

Here the chief worker (worker:0) hosts the native TCP store
(csrc/runtime/tcp_store.cpp) *at its own ClusterSpec address*; every other
task connects to it.  Ranks: workers first (0..W-1), then ps tasks.  Only
workers join the data-parallel group; ps tasks are control-plane members that
wait for the workers' done tokens (the shutdown protocol lr2.py:337-346 left
commented out).  The store also carries RCCL unique ids, barriers, heartbeats
and the chief-initialised flag (Supervisor semantics).
"""
from __future__ import annotations

import datetime
import json
import os
import threading
import time
from typing import Dict, List, Optional, Union

import torch.distributed as dist

from .. import _native


class ClusterSpec:
    """Drop-in for tf.train.ClusterSpec (dict of job -> list of "host:port")."""

    def __init__(self, cluster: Union[Dict[str, List[str]], "ClusterSpec", None] = None):
        if isinstance(cluster, ClusterSpec):
            cluster = cluster.as_dict()
        cluster = cluster or {}
        self._spec: Dict[str, List[str]] = {}
        for job, tasks in cluster.items():
            if isinstance(tasks, dict):  # {index: address}
                tasks = [tasks[k] for k in sorted(tasks)]
            if isinstance(tasks, str):
                tasks = [tasks]
            self._spec[str(job)] = [str(t) for t in tasks]

    @classmethod
    def from_json(cls, path: str) -> "ClusterSpec":
        with open(path) as f:
            return cls(json.load(f))

    def as_dict(self) -> Dict[str, List[str]]:
        return {k: list(v) for k, v in self._spec.items()}

    def as_cluster_def(self) -> Dict[str, List[str]]:
        return self.as_dict()

    @property
    def jobs(self) -> List[str]:
        return list(self._spec)

    def num_tasks(self, job_name: str) -> int:
        return len(self._spec.get(job_name, []))

    def task_indices(self, job_name: str) -> List[int]:
        return list(range(self.num_tasks(job_name)))

    def task_address(self, job_name: str, task_index: int) -> str:
        try:
            return self._spec[job_name][task_index]
        except (KeyError, IndexError):
            raise ValueError(f"no task {job_name}:{task_index} in cluster {self._spec}")

    def job_tasks(self, job_name: str) -> List[str]:
        return list(self._spec.get(job_name, []))

    # ------------------------------------------------------------- rank mapping
    def worker_job(self) -> str:
        return "worker" if "worker" in self._spec else ([j for j in self._spec if j != "ps"] or ["worker"])[0]

    def num_workers(self) -> int:
        return self.num_tasks(self.worker_job())

    def rank_of(self, job_name: str, task_index: int) -> int:
        wj = self.worker_job()
        if job_name == wj:
            return task_index
        base = self.num_workers()
        for j in self._spec:
            if j == wj:
                continue
            if j == job_name:
                return base + task_index
            base += self.num_tasks(j)
        raise ValueError(f"unknown job {job_name}")

    def total_tasks(self) -> int:
        return sum(len(v) for v in self._spec.values())

    def chief_address(self) -> str:
        return self.task_address(self.worker_job(), 0)

    def __eq__(self, other):
        return isinstance(other, ClusterSpec) and other.as_dict() == self.as_dict()

    def __repr__(self):
        return f"ClusterSpec({self._spec})"


def split_address(addr: str):
    addr = addr.split("://")[-1]
    host, _, port = addr.rpartition(":")
    return (host or "127.0.0.1"), int(port)


class NativeStore(dist.Store):
    """torch.distributed Store backed by the native TCP store (gloo bootstraps through it)."""

    def __init__(self, native, host: Optional[str] = None, port: Optional[int] = None, timeout_s: float = 300.0,
                 prefix: str = ""):
        # (torch's PrefixStore cannot wrap a Python store -- its clone() does
        # not dispatch back to Python -- so key prefixing is done here)
        super().__init__()
        self.s = native
        self._addr = (host, port, timeout_s)
        self.prefix = prefix

    def _k(self, key):
        return self.prefix + key

    def clone(self):
        # gloo opens extra store connections (one per async work thread)
        host, port, t = self._addr
        if host is None:
            return self
        return NativeStore(_native.load().TCPStore(host, port, False, t), host, port, t, self.prefix)

    def multi_get(self, keys):
        return [self.get(k) for k in keys]

    def multi_set(self, keys, values):
        for k, v in zip(keys, values):
            self.set(k, v)

    def append(self, key, value):
        while True:
            k = self._k(key)
            cur = self.s.get(k, 0.0) if self.s.check([k]) else b""
            new = cur + self._b(value)
            if self.s.compare_set(k, cur, new) == new:
                return

    def has_extended_api(self):
        return True

    @staticmethod
    def _b(v):
        if isinstance(v, str):
            return v.encode()
        return bytes(v)

    def set(self, key, value):
        self.s.set(self._k(key), self._b(value))

    def get(self, key):
        return self.s.get(self._k(key))

    def add(self, key, value):
        return self.s.add(self._k(key), int(value))

    def wait(self, keys, timeout=None):
        t = -1.0
        if isinstance(timeout, datetime.timedelta):
            t = timeout.total_seconds()
        self.s.wait([self._k(k) for k in keys], t)

    def check(self, keys):
        return self.s.check([self._k(k) for k in keys])

    def delete_key(self, key):
        return self.s.delete_key(self._k(key))

    def num_keys(self):
        return self.s.num_keys()

    def compare_set(self, key, expected, desired):
        return self.s.compare_set(self._k(key), self._b(expected), self._b(desired))


class Rendezvous:
    """Control plane of one task: store client (+ server on the chief)."""

    def __init__(self, cluster: ClusterSpec, job_name: str, task_index: int, timeout_s: float = 300.0,
                 bind_host: Optional[str] = None):
        self.cluster = cluster
        self.job_name = job_name
        self.task_index = int(task_index)
        self.rank = cluster.rank_of(job_name, task_index)
        self.world_size = cluster.total_tasks()
        self.num_workers = cluster.num_workers()
        self.is_worker = job_name == cluster.worker_job()
        self.is_chief = self.is_worker and self.task_index == 0
        host, port = split_address(cluster.chief_address())
        C = _native.load()
        if self.is_chief:
            self.store = C.TCPStore(bind_host if bind_host is not None else "0.0.0.0", port, True, timeout_s)
        else:
            self.store = C.TCPStore(host, port, False, timeout_s)
        self.timeout_s = timeout_s
        self._hb_thread = None
        self._hb_stop = threading.Event()
        self.store.set(f"task/{job_name}/{task_index}", str(os.getpid()).encode())

    # -------------------------------------------------------------- barriers etc
    def barrier(self, name: str, participants: Optional[int] = None):
        self.store.barrier(name, participants or self.world_size, self.timeout_s)

    def worker_barrier(self, name: str):
        self.store.barrier("w/" + name, self.num_workers, self.timeout_s)

    def publish(self, key: str, value: bytes):
        self.store.set(key, value)

    def fetch(self, key: str, timeout: float = -1.0) -> bytes:
        return self.store.get(key, timeout)

    # -------------------------------------------------------------- done tokens
    def signal_done(self):
        """Worker -> ps shutdown token (the commented protocol of lr2.py:337-346)."""
        self.store.set(f"done/{self.job_name}/{self.task_index}", b"1")

    def wait_all_workers_done(self, timeout: float = -1.0, poll: float = 0.5,
                              on_dead=None):
        keys = [f"done/{self.cluster.worker_job()}/{i}" for i in range(self.num_workers)]
        start = time.time()
        while True:
            if self.store.check(keys):
                return True
            if on_dead is not None:
                dead = self.dead_workers()
                if dead:
                    on_dead(dead)
            if 0 <= timeout < time.time() - start:
                return False
            time.sleep(poll)

    # -------------------------------------------------------------- heartbeats
    def start_heartbeat(self, interval: float = 1.0):
        if self._hb_thread is not None:
            return

        def beat():
            key = f"hb/{self.job_name}/{self.task_index}"
            while not self._hb_stop.wait(interval):
                try:
                    self.store.set(key, repr(time.time()).encode())
                except Exception:
                    return

        self.store.set(f"hb/{self.job_name}/{self.task_index}", repr(time.time()).encode())
        self._hb_thread = threading.Thread(target=beat, daemon=True, name="dtf-heartbeat")
        self._hb_thread.start()

    def dead_workers(self, stale_s: float = 10.0) -> List[int]:
        now = time.time()
        dead = []
        wj = self.cluster.worker_job()
        for i in range(self.num_workers):
            key = f"hb/{wj}/{i}"
            if not self.store.check([key]):
                continue
            if self.store.check([f"done/{wj}/{i}"]):
                continue
            t = float(self.store.get(key, 1.0).decode())
            if now - t > stale_s:
                dead.append(i)
        return dead

    def stop_heartbeat(self, wait_s: float = 2.0):
        """Stop beating and wait for the thread: a daemon thread still inside a
        native store call while the interpreter finalises can abort the process
        (a task that left must not beat into a store the chief is closing)."""
        self._hb_stop.set()
        t = self._hb_thread
        if t is not None and t.is_alive() and t is not threading.current_thread():
            t.join(wait_s)

    def close(self):
        self.stop_heartbeat()
        try:
            self.store.close()
        except Exception:
            pass
