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

Partitioned (row-sharded) variables -- lr2.py's ps-held `W[F, 1]` trained by
`embedding_lookup_sparse` + ScatterSub on the ps -- use `HogwildTable`: every
rank's shard (row r on rank r % W at local row r // W) is mapped into every
rank (GPU: IPC peer buffers, csrc/kernels/hogwild.hip row gather / scatter-SGD
over xGMI; CPU: one /dev/shm file per shard), so a worker reads its batch's
unique rows straight from their owners and applies its sparse update into
them without waiting for any other worker -- no collective on the step.

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


class HogwildTable:
    """A row-sharded table (parallel/sharded_embedding.ShardedEmbedding) shared
    for asynchronous sparse SGD.  Collective to construct; `lookup` /
    `scatter_sgd` are rank-local and never wait for another rank.  The table's
    own shard (`table.local`) is re-homed into the shared mapping, so
    checkpoints, `full_table()` and evaluation keep seeing the live values."""

    def __init__(self, table, world, use_locking: bool = False):
        self.table = table
        self.world = world
        self.W = world.world_size if world is not None else 1
        self.rank = world.rank if world is not None else 0
        self.locking = bool(use_locking)
        self.D = table.dim
        self.device = table.device
        self.kind = "local"
        self._ipc = None
        self._maps = []
        if self.W > 1 and self.device.type == "cuda":
            self._open_ipc()
        elif self.W > 1:
            self._open_shm()
        if self.W > 1:
            world.barrier()

    def _rows_of(self, r: int) -> int:
        F = self.table.num_rows
        return (F - r + self.W - 1) // self.W if r < F else 0

    def _open_ipc(self):
        from .. import _native
        from .world import open_peer_buffers

        C = _native.load()
        n_max = (self.table.num_rows + self.W - 1) // self.W
        self._ipc = open_peer_buffers(C, 4 * max(1, n_max * self.D), self.world)
        own = self._ipc.tensor(0, self._rows_of(self.rank) * self.D, 0).view(-1, self.D)
        with torch.no_grad():
            own.copy_(self.table.local)
        self.table.local = own
        self._C = C
        self._shards = int(self._ipc.table_ptr())
        torch.cuda.synchronize(self.device)
        self.kind = "ipc"

    def _open_shm(self):
        n = self._rows_of(self.rank) * self.D
        fd, path = tempfile.mkstemp(prefix=f"dtf_hogtab_{self.rank}_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
        os.ftruncate(fd, 4 * max(1, n))
        os.close(fd)
        paths = self.world.all_gather_object(path)
        self._files, self._shards_t = [], []
        for r, pth in enumerate(paths):
            f = open(pth, "r+b")
            nr = self._rows_of(r) * self.D
            mm = mmap.mmap(f.fileno(), 4 * max(1, nr))
            self._files.append(f)
            self._maps.append(mm)
            self._shards_t.append(torch.from_numpy(np.frombuffer(mm, dtype=np.float32, count=nr)).view(-1, self.D))
        with torch.no_grad():
            self._shards_t[self.rank].copy_(self.table.local)
        self.table.local = self._shards_t[self.rank]
        self.world.barrier()           # every rank mapped every shard: the names can go
        os.unlink(path)
        self.kind = "shm"

    def lookup(self, ids: torch.Tensor):
        """(rows [U, D] as the owners hold them now, inverse, unique ids)."""
        ids = ids.to(self.device).long()
        uniq, inverse = torch.unique(ids, return_inverse=True)
        if self.kind == "ipc":
            rows = torch.empty((uniq.numel(), self.D), dtype=torch.float32, device=self.device)
            self._C.hogwild_gather_rows(uniq.contiguous(), self._shards, self.W, rows)
        elif self.kind == "shm":
            rows = torch.empty((uniq.numel(), self.D), dtype=torch.float32)
            owner, local = uniq % self.W, uniq // self.W
            for r in range(self.W):
                m = owner == r
                if bool(m.any()):
                    rows[m] = self._shards_t[r].index_select(0, local[m])
        else:
            rows = self.table.local.index_select(0, uniq)
        return rows, inverse, uniq

    def scatter_sgd(self, uniq: torch.Tensor, grads: torch.Tensor, lr: float):
        """rows[uniq] -= lr * grads on their owners' shards, no waiting (use_locking:
        per-element CAS on GPU, an advisory lock per shard file on CPU)."""
        g = grads.float().reshape(-1, self.D).contiguous()
        if uniq.numel() == 0:
            return
        with torch.no_grad():
            if self.kind == "ipc":
                self._C.hogwild_scatter_sgd(uniq.contiguous(), g, self._shards, self.W, float(lr), self.locking)
            elif self.kind == "shm":
                owner, local = uniq % self.W, uniq // self.W
                for r in range(self.W):
                    m = owner == r
                    if not bool(m.any()):
                        continue
                    if self.locking:
                        fcntl.lockf(self._files[r], fcntl.LOCK_EX)
                    try:
                        self._shards_t[r].index_add_(0, local[m], g[m], alpha=-float(lr))
                    finally:
                        if self.locking:
                            fcntl.lockf(self._files[r], fcntl.LOCK_UN)
            else:
                self.table.local.index_add_(0, uniq, g, alpha=-float(lr))

    def close(self):
        """Give the table a private copy of its shard again and unmap the others."""
        if self.kind == "local":
            return
        with torch.no_grad():
            own = self.table.local.clone()
        if self.kind == "ipc":
            torch.cuda.synchronize(self.device)
            self.world.barrier()        # nobody still reads / writes a peer shard
            self.table.local = own
            self._ipc.close()
            self._ipc = None
        else:
            self.world.barrier()
            self.table.local = own
            self._shards_t = []
            for mm in self._maps:
                mm.close()
            for f in self._files:
                f.close()
            self._maps, self._files = [], []
        self.kind = "local"
