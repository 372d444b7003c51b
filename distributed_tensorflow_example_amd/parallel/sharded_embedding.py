"""Row-sharded embedding tables: the parameter-server role, one shard per GPU.

Reference: the LR weight `W[F, 1]` (F = 4.7M, 1e9 in product,
lr2.py:384 / run_lr2.sh:56) lives on ps0 via replica_device_setter
(lr2.py:359-361); each step the worker sends the batch's unique ids, the ps
gathers rows, the worker returns IndexedSlices gradients that the ps
scatter-applies.  The commented Wide&Deep tower
(lr2_debug.py:423-428) adds a [F, 128] table the same way.

MI355X design: row r lives on rank r % W at local row r // W (288 GB of
HBM per GPU holds a 1e9 x 1 fp32 shard 8x over).  Per step:

  lookup:  dedup ids (torch.unique) -> bucket by owner -> all-to-all of ids
           -> owners gather rows -> all-to-all back            (RCCL / gloo)
  combine: the CSR bag kernel (ops.embedding_bag) runs over the gathered
           [U, D] block with ids remapped to 0..U-1
  update:  bag backward into a dense [U, D] gradient -> all-to-all to owners
           -> owners apply SGD with the fused scatter kernel

Each row has exactly one owner, so there is no replica drift and no
all-reduce of a dense F x D gradient.  Initial values are a counter-based
(Philox4x32-10) normal of the *global* element index, generated on the device
by one kernel, so a table is bit-identical for any world size.
Checkpoints store the table as a TF partitioned variable (contiguous
fixed_size_partitioner slices, see ckpt/__init__.py).
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import ops
from .world import World, get_world

class LookupCtx:
    """Routing of one batch.  Dynamic: exact per-peer counts (host lists in
    send/recv), `order` sorts uniq by owner.  Static: every peer gets `cap`
    slots (a capacity configured identically on all ranks, >= the ids of any
    batch, so no bucket can overflow), `order` holds each unique id's slot
    (dest, -1 for padding) and uniq / recv_local carry -1 padding -- no host
    read-back, every shape fixed by the batch shape and the capacity."""
    __slots__ = ("uniq", "inverse", "order", "send", "recv", "recv_local", "static", "n")

    def __init__(self, uniq, inverse, order, send, recv, recv_local, static=False, n=0):
        self.uniq, self.inverse, self.order = uniq, inverse, order
        self.send, self.recv, self.recv_local = send, recv, recv_local
        self.static, self.n = static, n


class ShardedEmbedding:
    def __init__(self, num_rows: int, dim: int = 1, world: Optional[World] = None, init_std: float = 1.0,
                 seed: int = 0, device=None, name: str = "embedding", zero_init: bool = False,
                 capacity: Optional[int] = None):
        self.world = world or get_world()
        self.W = self.world.world_size
        self.rank = self.world.rank
        self.num_rows, self.dim, self.name = int(num_rows), int(dim), name
        self.capacity = capacity          # ids per batch bound (same on every rank) -> static routing
        self.device = torch.device(device) if device is not None else self.world.device
        n_local = (self.num_rows - self.rank + self.W - 1) // self.W if self.rank < self.num_rows else 0
        self.local = torch.empty((n_local, self.dim), dtype=torch.float32, device=self.device)
        with torch.no_grad():
            if zero_init:
                self.local.zero_()
            else:
                # local row i is global row i*W + rank: one counter-based
                # Philox kernel over the shard (csrc/kernels/random.hip)
                ops.philox_normal_(self.local, self.W, self.rank, seed, 0.0, init_std)

    # ------------------------------------------------------------------ exchange
    def route(self, ids: torch.Tensor, capacity: Optional[int] = None) -> LookupCtx:
        """Dedup `ids` and send each owner the unique ids it serves (no rows yet).

        The context depends only on the ids and the row partition, so tables
        with the same row count and world share it (`lookup_shared`).
        `capacity`: ids-per-batch bound configured identically on every rank ->
        the device-resident static exchange (no host read-back); without it
        (W > 1) the exact per-peer counts are exchanged and read on the host."""
        ids = ids.to(self.device).long()
        N = ids.numel()
        capacity = self.capacity if capacity is None else capacity
        if N > 0 and (self.W == 1 or (capacity is not None and self.W <= _max_route_world())):
            if self.W > 1 and N > capacity:
                raise ValueError(f"{self.name}: batch has {N} ids, above the routing capacity {capacity}")
            return self._route_static(ids, int(capacity) if capacity is not None else N)
        if ids.is_cuda and 0 < N and self.num_rows < 2 ** 31:
            # one int32 radix sort serves both the dedup and (handed over to
            # ops) the sorted-segment backward of every bag over these ids
            sids, perm = torch.sort(ids.to(torch.int32))
            uniq32, inv_sorted = torch.unique_consecutive(sids, return_inverse=True)
            uniq = uniq32.long()
            inverse = torch.empty_like(ids)
            inverse[perm] = inv_sorted
            ops.register_sorted_ids(inverse, inv_sorted, perm)
        else:
            uniq, inverse = torch.unique(ids, return_inverse=True)
        if self.W == 1:
            return LookupCtx(uniq, inverse, None, None, None, uniq)
        owner = uniq % self.W
        order = torch.argsort(owner, stable=True)
        uniq_sorted = uniq[order]
        send = torch.bincount(owner, minlength=self.W)
        recv = torch.empty_like(send)
        self.world.all_to_all(send, [1] * self.W, recv, [1] * self.W)
        send_l, recv_l = send.tolist(), recv.tolist()
        recv_ids = torch.empty(sum(recv_l), dtype=torch.int64, device=self.device)
        self.world.all_to_all(uniq_sorted, send_l, recv_ids, recv_l)
        return LookupCtx(uniq, inverse, order, send_l, recv_l, recv_ids // self.W)

    def _route_static(self, ids: torch.Tensor, cap: int) -> LookupCtx:
        """Device-resident routing: radix sort + one dedup/bucketing kernel
        (csrc/kernels/sparse_route.hip) + an equal-split all-to-all of `cap` id
        slots per peer.  Nothing is read back to the host."""
        N, W = ids.numel(), self.W
        small = self.num_rows < 2 ** 31
        sids, perm = torch.sort(ids.to(torch.int32) if small else ids)
        if ids.is_cuda:
            inv_sorted, inverse, uniq, dest, send, _count = ops._C().sparse_route(sids.contiguous(), perm, W, cap)
            ops.register_sorted_ids(inverse, inv_sorted, perm)
        else:
            inv_sorted, inverse, uniq, dest, send = _route_static_torch(sids, perm, W, cap)
        if W == 1:
            return LookupCtx(uniq, inverse, None, None, None, uniq, static=True, n=N)
        recv = torch.empty(W * cap, dtype=torch.int64, device=self.device)
        self.world.all_to_all(send, [cap] * W, recv, [cap] * W)
        recv_local = torch.where(recv >= 0, recv // W, torch.full_like(recv, -1))
        return LookupCtx(uniq, inverse, dest.long(), [cap] * W, [cap] * W, recv_local, static=True, n=cap)

    def lookup(self, ids: torch.Tensor):
        """rows [U, D] for the unique ids of `ids`, plus the routing context."""
        ctx = self.route(ids)
        return lookup_shared([self], ctx)[0], ctx

    def apply_sgd(self, ctx: LookupCtx, grad_rows: torch.Tensor, lr: float):
        """local[owner rows] -= lr * grad (grad_rows aligned with ctx.uniq)."""
        apply_sgd_shared([self], ctx, [grad_rows], [lr])

    def _sgd_local(self, ctx: LookupCtx, g: torch.Tensor, lr: float):
        n = g.shape[0]
        if n == 0:
            return
        offs = torch.arange(n + 1, dtype=torch.int64, device=self.device)
        with torch.no_grad():
            ops.embedding_bag_sgd_(self.local, ctx.recv_local, offs, None, g, float(lr))

    # ------------------------------------------------------------------ bags
    def bag_forward(self, ids, offsets, weights=None, mode: str = "sum"):
        """embedding_lookup_sparse over the sharded table -> ([B, D], ctx)."""
        rows, ctx = self.lookup(ids)
        rows = rows.detach().requires_grad_(True)
        out = ops.embedding_bag(rows, ctx.inverse, offsets.to(self.device).long(),
                                None if weights is None else weights.to(self.device).float(), mode)
        return out, (rows, ctx)

    def bag_backward_sgd(self, state, lr: float):
        rows, ctx = state
        g = rows.grad if rows.grad is not None else torch.zeros_like(rows)
        self.apply_sgd(ctx, g, lr)

    # ------------------------------------------------------------------ checkpoint
    def full_table(self) -> torch.Tensor:
        """Gather the whole table on every rank (small tables / tests only)."""
        if self.W == 1:
            return self.local.detach().clone()
        n_max = (self.num_rows + self.W - 1) // self.W
        pad = torch.zeros((n_max, self.dim), dtype=torch.float32, device=self.device)
        pad[: self.local.shape[0]] = self.local
        allp = torch.empty((self.W * n_max, self.dim), dtype=torch.float32, device=self.device)
        self.world.all_gather(pad, allp)
        allp = allp.view(self.W, n_max, self.dim)
        out = torch.empty((self.num_rows, self.dim), dtype=torch.float32, device=self.device)
        for r in range(self.W):
            n_r = (self.num_rows - r + self.W - 1) // self.W
            out[r::self.W] = allp[r, :n_r]
        return out

    def shard_name(self) -> str:
        return f"{self.name}/part_{self.rank}"

    def load_full(self, table: torch.Tensor):
        with torch.no_grad():
            self.local.copy_(table.to(self.device)[self.rank::self.W])


def _check_shared(tables):
    t0 = tables[0]
    for t in tables[1:]:
        if t.num_rows != t0.num_rows or t.world is not t0.world:
            raise ValueError("tables sharing one routing context need the same row count and world")


def lookup_shared(tables, ctx: LookupCtx):
    """Rows of every table for ctx.uniq with ONE row all-to-all: owners gather
    each table's rows side by side ([n, sum D]) so W&D's wide and deep tables
    (same ids, same partition) pay one dedup, one id exchange and one row
    exchange per step instead of two of each."""
    _check_shared(tables)
    t0 = tables[0]
    if t0.W == 1:
        idx = ctx.uniq.clamp_min(0) if ctx.static else ctx.uniq     # padding slots read row 0, never used
        return [t.local.index_select(0, idx) for t in tables]
    dims = [t.dim for t in tables]
    src = ctx.recv_local.clamp_min(0) if ctx.static else ctx.recv_local
    served = torch.cat([t.local.index_select(0, src) for t in tables], 1) if len(tables) > 1 else \
        t0.local.index_select(0, src)
    got = torch.empty((sum(ctx.send), sum(dims)) if ctx.static else (ctx.uniq.numel(), sum(dims)),
                      dtype=torch.float32, device=t0.device)
    t0.world.all_to_all(served.contiguous(), ctx.recv, got, ctx.send)
    if ctx.static:
        rows = got.index_select(0, ctx.order.clamp_min(0))          # slot of each unique id
    else:
        rows = torch.empty_like(got)
        rows[ctx.order] = got
    return list(rows.split(dims, 1)) if len(tables) > 1 else [rows]


def apply_sgd_shared(tables, ctx: LookupCtx, grads, lrs):
    """Sparse SGD on every table; the gradients travel to the owners in ONE
    all-to-all (columns side by side, same routing as `lookup_shared`)."""
    _check_shared(tables)
    t0 = tables[0]
    gs = [g.float().reshape(-1, t.dim) for t, g in zip(tables, grads)]
    if t0.W > 1:
        g = torch.cat(gs, 1) if len(gs) > 1 else gs[0]
        if ctx.static:
            valid = (ctx.order >= 0).unsqueeze(1).to(g.dtype)
            g_sorted = torch.zeros((sum(ctx.send), g.shape[1]), dtype=torch.float32, device=t0.device)
            g_sorted.index_add_(0, ctx.order.clamp_min(0), g * valid)   # padding adds 0
        else:
            g_sorted = g[ctx.order].contiguous()
        recv_g = torch.empty((sum(ctx.recv), g.shape[1]), dtype=torch.float32, device=t0.device)
        t0.world.all_to_all(g_sorted, ctx.send, recv_g, ctx.recv)
        gs = list(recv_g.split([t.dim for t in tables], 1))
    for t, g, lr in zip(tables, gs, lrs):
        t._sgd_local(ctx, g.contiguous(), lr)


def _max_route_world() -> int:
    try:
        return ops._C().route_max_world()
    except Exception:       # CPU-only build without the extension: the torch emulation has no limit
        return 1 << 30


def _route_static_torch(sids: torch.Tensor, perm: torch.Tensor, W: int, cap: int):
    """CPU emulation of csrc/kernels/sparse_route.hip (same outputs)."""
    N = sids.numel()
    dev = sids.device
    flag = torch.ones(N, dtype=torch.bool, device=dev)
    flag[1:] = sids[1:] != sids[:-1]
    inv_sorted = (torch.cumsum(flag.to(torch.int64), 0) - 1).to(torch.int32)
    inverse = torch.empty(N, dtype=torch.int64, device=dev)
    inverse[perm] = inv_sorted.long()
    u = sids[flag].long()
    U = u.numel()
    uniq = torch.full((N,), -1, dtype=torch.int64, device=dev)
    uniq[:U] = u
    dest = torch.full((N,), -1, dtype=torch.int32, device=dev)
    send = torch.full((W * cap,), -1, dtype=torch.int64, device=dev)
    if W > 1 and U:
        owner = u % W
        counts = torch.bincount(owner, minlength=W)
        start = torch.cumsum(counts, 0) - counts
        order = torch.argsort(owner, stable=True)          # id order within each owner
        pos = torch.empty(U, dtype=torch.int64, device=dev)
        pos[order] = torch.arange(U, device=dev) - start[owner[order]]
        d = owner * cap + pos
        dest[:U] = d.to(torch.int32)
        send[d] = u
    return inv_sorted, inverse, uniq, dest, send
