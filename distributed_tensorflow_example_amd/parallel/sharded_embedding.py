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
normal of the *global* row id, so a table is bit-identical for any world size.
Checkpoints store the table as a TF partitioned variable (contiguous
fixed_size_partitioner slices, see ckpt/__init__.py).
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from .. import ops
from .world import World, get_world

_M1 = 0x9E3779B97F4A7C15 - (1 << 64)   # as signed int64
_M2 = 0xBF58476D1CE4E5B9 - (1 << 64)
_M3 = 0x94D049BB133111EB - (1 << 64)


def _mix(x: torch.Tensor) -> torch.Tensor:
    """splitmix64 finaliser on int64 tensors (wrap-around arithmetic)."""
    x = x + _M1
    x = (x ^ ((x >> 30) & 0x3FFFFFFFF)) * _M2
    x = (x ^ ((x >> 27) & 0x1FFFFFFFFF)) * _M3
    return x ^ ((x >> 31) & 0x1FFFFFFFF)


def counter_normal(rows: torch.Tensor, dim: int, seed: int, std: float = 1.0) -> torch.Tensor:
    """N(0, std^2) values for (global row, col), independent of sharding."""
    col = torch.arange(dim, device=rows.device, dtype=torch.int64)
    key = rows.long().unsqueeze(1) * dim + col + (int(seed) << 40)
    a = _mix(key)
    b = _mix(a ^ 0x5851F42D4C957F2D)
    u1 = ((a >> 11) & ((1 << 53) - 1)).double().add_(0.5).mul_(1.0 / (1 << 53))
    u2 = ((b >> 11) & ((1 << 53) - 1)).double().mul_(1.0 / (1 << 53))
    z = torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(2 * math.pi * u2)
    return (z * std).float()


class LookupCtx:
    __slots__ = ("uniq", "inverse", "order", "send", "recv", "recv_local")

    def __init__(self, uniq, inverse, order, send, recv, recv_local):
        self.uniq, self.inverse, self.order = uniq, inverse, order
        self.send, self.recv, self.recv_local = send, recv, recv_local


class ShardedEmbedding:
    def __init__(self, num_rows: int, dim: int = 1, world: Optional[World] = None, init_std: float = 1.0,
                 seed: int = 0, device=None, name: str = "embedding", zero_init: bool = False,
                 init_chunk_rows: int = 1 << 24):
        self.world = world or get_world()
        self.W = self.world.world_size
        self.rank = self.world.rank
        self.num_rows, self.dim, self.name = int(num_rows), int(dim), name
        self.device = torch.device(device) if device is not None else self.world.device
        n_local = (self.num_rows - self.rank + self.W - 1) // self.W if self.rank < self.num_rows else 0
        self.local = torch.empty((n_local, self.dim), dtype=torch.float32, device=self.device)
        with torch.no_grad():
            if zero_init:
                self.local.zero_()
            else:
                for s in range(0, n_local, init_chunk_rows):
                    e = min(n_local, s + init_chunk_rows)
                    grow = torch.arange(s, e, device=self.device, dtype=torch.int64) * self.W + self.rank
                    self.local[s:e] = counter_normal(grow, self.dim, seed, init_std)

    # ------------------------------------------------------------------ exchange
    def route(self, ids: torch.Tensor) -> LookupCtx:
        """Dedup `ids` and send each owner the unique ids it serves (no rows yet).

        The context depends only on the ids and the row partition, so tables
        with the same row count and world share it (`lookup_shared`)."""
        ids = ids.to(self.device).long()
        if ids.is_cuda and 0 < ids.numel() and self.num_rows < 2 ** 31:
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
        return [t.local.index_select(0, ctx.uniq) for t in tables]
    dims = [t.dim for t in tables]
    served = torch.cat([t.local.index_select(0, ctx.recv_local) for t in tables], 1) if len(tables) > 1 else \
        t0.local.index_select(0, ctx.recv_local)
    got = torch.empty((ctx.uniq.numel(), sum(dims)), dtype=torch.float32, device=t0.device)
    t0.world.all_to_all(served.contiguous(), ctx.recv, got, ctx.send)
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
        g_sorted = g[ctx.order].contiguous()
        recv_g = torch.empty((sum(ctx.recv), g.shape[1]), dtype=torch.float32, device=t0.device)
        t0.world.all_to_all(g_sorted, ctx.send, recv_g, ctx.recv)
        gs = list(recv_g.split([t.dim for t in tables], 1))
    for t, g, lr in zip(tables, gs, lrs):
        t._sgd_local(ctx, g.contiguous(), lr)
