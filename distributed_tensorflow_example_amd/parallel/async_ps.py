"""Asynchronous (Hogwild) parameter-server training: the reference's default
update rule.

example.py:64-118 (and lr2.py) build a between-graph replicated graph under
`replica_device_setter` and train it with a plain `GradientDescentOptimizer`:
every worker reads the ps-held variables, computes the gradient of its own
batch and applies `var -= lr * grad` on the ps with no coordination
(`use_locking=False`), and `global_step` counts every worker's step
(the synchronous `SyncReplicasOptimizer` variant is commented out there).
This repo's default is synchronous data parallelism (BASELINE north star);
`HogwildStore` provides the asynchronous mode when asked for
(`DTF_UPDATE_MODE=async`, or `Optimizer(..., update_mode="async")`).

MI355X-first layout -- no parameter-server process on the data path:

* GPU workers of one node: the "ps variables" are ONE flat fp32 buffer (plus a
  64-bit global-step counter) in the device memory of rank 0, allocated
  uncached and IPC-mapped into every rank (csrc/comm/ipc_peer.cpp).  Each step
  a worker pulls it (system-scope loads over xGMI), runs forward + backward on
  its own GPU, and applies its SGD update straight into the shared buffer with
  one kernel (csrc/kernels/hogwild.hip: read-modify-write per element, or a
  CAS loop with `use_locking=True`) that also bumps the shared global step.
* CPU workers (gloo, tests, the 1-ps-plus-workers plumbing config): the same
  flat buffer in a /dev/shm file mapped by every rank; updates under an
  advisory file lock when `use_locking=True`, racy otherwise.
* world_size 1: the local parameters are the store.

The ps tasks stay control-plane members (done tokens, `server.join()`), as in
the synchronous mode.
"""
from __future__ import annotations

import fcntl
import mmap
import os
import tempfile
from typing import List, Optional

import numpy as np
import torch

_COUNTER_PAD = 32   # floats behind the parameters: the 8-byte step counter at the next 64-B boundary


def update_mode(explicit: Optional[str] = None) -> str:
    """'sync' (default: all-reduce data parallelism) or 'async' (Hogwild ps)."""
    m = (explicit or os.environ.get("DTF_UPDATE_MODE", "sync")).lower()
    if m not in ("sync", "async"):
        raise ValueError(f"update mode must be 'sync' or 'async', not {m!r}")
    return m


class HogwildStore:
    """Shared flat parameter buffer + global-step counter for asynchronous SGD.

    Collective to construct (every rank of `world`); `pull` / `sgd_step` are
    rank-local and never wait for another rank."""

    def __init__(self, params: List[torch.Tensor], world, use_locking: bool = False):
        self.params = list(params)
        self.world = world
        self.locking = bool(use_locking)
        self.sizes = [p.numel() for p in self.params]
        self.n = int(sum(self.sizes))
        self.device = self.params[0].device
        self.flat_p = torch.zeros(self.n, dtype=torch.float32, device=self.device)
        self.flat_g = torch.zeros(self.n, dtype=torch.float32, device=self.device)
        self._pv = self._views(self.flat_p)
        self._gv = self._views(self.flat_g)
        self.kind = "local"
        self._ipc = None
        self._shm = None
        self._lockf = None
        ws = world.world_size if world is not None else 1
        if ws > 1 and self.device.type == "cuda":
            self._open_ipc()
        elif ws > 1:
            self._open_shm()
        self._init_from_chief()

    # ------------------------------------------------------------------ setup
    def _views(self, flat):
        out, off = [], 0
        for p, n in zip(self.params, self.sizes):
            out.append(flat[off:off + n].view_as(p))
            off += n
        return out

    def _open_ipc(self):
        from .. import _native
        from .world import open_peer_buffers

        C = _native.load()
        nbytes = 4 * (self.n + _COUNTER_PAD)
        self._ipc = open_peer_buffers(C, nbytes, self.world)
        self._C = C
        self._shared = int(self._ipc.peer_ptr(0))                 # rank 0 hosts the variables
        self._counter = self._shared + 4 * (self.n + (-self.n) % 16)
        self._gstep_dev = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.kind = "ipc"

    def _open_shm(self):
        w = self.world
        path = None
        if w.rank == 0:
            fd, path = tempfile.mkstemp(prefix="dtf_hogwild_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
            os.ftruncate(fd, 4 * (self.n + _COUNTER_PAD))
            os.close(fd)
        path = w.broadcast_object(path, src=0)
        f = open(path, "r+b")
        self._mm = mmap.mmap(f.fileno(), 4 * (self.n + _COUNTER_PAD))
        self._lockf = f
        arr = np.frombuffer(self._mm, dtype=np.float32)
        self._shared_t = torch.from_numpy(arr[:self.n])
        self._counter_np = np.frombuffer(self._mm, dtype=np.int64, count=1, offset=4 * (self.n + (-self.n) % 16))
        w.barrier()                     # everyone mapped it: the name can go
        if w.rank == 0:
            os.unlink(path)
        self._shm = path
        self.kind = "shm"

    def _init_from_chief(self):
        """The chief's (already broadcast) values become the ps variables; global step 0."""
        w = self.world
        if self.kind == "local":
            return
        if w.rank == 0:
            with torch.no_grad():
                for v, p in zip(self._pv, self.params):
                    v.copy_(p)
            if self.kind == "ipc":
                self._ipc_write_all()
            else:
                self._shared_t.copy_(self.flat_p)
                self._counter_np[0] = 0
        if self.kind == "ipc":
            torch.cuda.synchronize(self.device)
        w.barrier()

    def _ipc_write_all(self):
        # rank 0 owns the buffer: write the initial values through its own mapping
        self._ipc.tensor(0, self.n, 0).copy_(self.flat_p)
        self._C.hogwild_counter(self._counter, self._gstep_dev, set=0, do_set=True)

    # ------------------------------------------------------------------ steps
    def pull(self):
        """Local parameters <- current ps variables (before a forward)."""
        if self.kind == "local":
            return
        with torch.no_grad():
            if self.kind == "ipc":
                self._C.hogwild_pull(self._shared, self.flat_p)
            else:
                self.flat_p.copy_(self._shared_t)
            for v, p in zip(self._pv, self.params):
                p.copy_(v)

    def sgd_step(self, grads: List[Optional[torch.Tensor]], lr: float) -> int:
        """Apply `var -= lr * grad` to the ps variables (no waiting for other
        workers), refresh the local copy with the values written, return the
        global step after this update (every worker's steps count)."""
        with torch.no_grad():
            for v, g in zip(self._gv, grads):
                if g is None:
                    v.zero_()
                else:
                    v.copy_(g)
            if self.kind == "local":
                self.flat_p.copy_(torch.cat([p.reshape(-1) for p in self.params]))
                self.flat_p.sub_(self.flat_g, alpha=lr)
                for v, p in zip(self._pv, self.params):
                    p.copy_(v)
                self._local_steps = getattr(self, "_local_steps", 0) + 1
                return self._local_steps
            if self.kind == "ipc":
                self._C.hogwild_sgd(self._shared, self.flat_g, self.flat_p, float(lr), self.locking, self._counter,
                                    self._gstep_dev)
                gstep = int(self._gstep_dev.item())
            else:
                if self.locking:
                    fcntl.lockf(self._lockf, fcntl.LOCK_EX)
                try:
                    self._shared_t.sub_(self.flat_g, alpha=lr)
                    self.flat_p.copy_(self._shared_t)
                finally:
                    if self.locking:
                        fcntl.lockf(self._lockf, fcntl.LOCK_UN)
                fcntl.lockf(self._lockf, fcntl.LOCK_EX, 8, 4 * (self.n + (-self.n) % 16))
                try:
                    self._counter_np[0] += 1
                    gstep = int(self._counter_np[0])
                finally:
                    fcntl.lockf(self._lockf, fcntl.LOCK_UN, 8, 4 * (self.n + (-self.n) % 16))
            for v, p in zip(self._pv, self.params):
                p.copy_(v)
        return gstep

    def global_step(self) -> int:
        if self.kind == "ipc":
            self._C.hogwild_counter(self._counter, self._gstep_dev)
            return int(self._gstep_dev.item())
        if self.kind == "shm":
            return int(self._counter_np[0])
        return getattr(self, "_local_steps", 0)

    def close(self):
        if self._ipc is not None:
            torch.cuda.synchronize(self.device)
            self.world.barrier()         # nobody still writes into rank 0's buffer
            self._ipc.close()
            self._ipc = None
        if self._shm is not None:
            self._counter_np = None
            self._shared_t = None
            self._mm = None
            self._lockf.close()
            self._shm = None
