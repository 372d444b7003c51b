"""Distributed TF-format checkpoints: every rank writes its own data shard.

A TF V2 bundle may span N data files (`prefix.data-0000k-of-0000N`) with one
merged `prefix.index`.  Row-sharded tables (the parameter-server part of the
model, parallel.sharded_embedding: row r on rank r % W) are saved the way TF's
Saver saves a PartitionedVariable: P contiguous row partitions
(tf.fixed_size_partitioner sizing), each written as a slice -- data under the
EncodeTensorNameSlice key, a TensorSliceProto in the full-name entry
(compat/saver.py, csrc/runtime/tf_bundle.cpp).  Partition k is assembled on
rank k % W by one all-to-all of the rows it needs (no gather of a 1e9-row
table onto one host) and written into that rank's shard in parallel; the chief
merges the per-shard index tables (native `bundle_merge_shard_indexes`, which
concatenates the slice lists of one variable) and updates the `checkpoint`
state file.  Replicated tensors are written once, by the chief.

Restore streams one slice at a time and keeps the rows the rank owns, so a
checkpoint written by any world size / partition count -- or a plain full
entry from an unpartitioned TF variable -- loads on any world size.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Union

import torch

from .. import _native
from ..compat.saver import (iter_slices, latest_checkpoint, partition_extents, read_bundle_index, read_tensor,
                            update_checkpoint_state, write_bundle)
from ..parallel.sharded_embedding import ShardedEmbedding
from ..parallel.world import World, get_world

__all__ = ["save_sharded", "restore_sharded", "restore_table", "gather_partitions", "gather_rows",
           "latest_checkpoint", "read_tensor", "read_bundle_index", "partition_extents"]


def _owned(rank: int, W: int, lo: int, hi: int):
    """Local index range [i0, i1) of the rows in [lo, hi) that `rank` owns."""
    i0 = max(0, -(-(lo - rank) // W))
    i1 = max(0, -(-(hi - rank) // W))
    return i0, max(i0, i1)


def gather_rows(table: ShardedEmbedding, lo: int, hi: int, dst: int) -> Optional[torch.Tensor]:
    """Collective: rows [lo, hi) of the modulo-sharded table, assembled on
    rank `dst` (None elsewhere).  One uneven all-to-all in which only `dst`
    receives."""
    W, r = table.W, table.rank
    if W == 1:
        return table.local[lo:hi]
    counts = [_owned(s, W, lo, hi) for s in range(W)]
    i0, i1 = counts[r]
    send = [0] * W
    send[dst] = i1 - i0
    recv_counts = [b - a for a, b in counts] if r == dst else [0] * W
    recv = torch.empty((sum(recv_counts), table.dim), dtype=table.local.dtype, device=table.device)
    table.world.all_to_all(table.local[i0:i1].contiguous(), send, recv, recv_counts)
    if r != dst:
        return None
    out = torch.empty((hi - lo, table.dim), dtype=recv.dtype, device=recv.device)
    off = 0
    for s, (a, b) in enumerate(counts):
        if b > a:
            first = s + a * W - lo
            out[first:first + (b - a) * W:W] = recv[off:off + b - a]
            off += b - a
    return out


def gather_partitions(table: ShardedEmbedding, name: str, full_shape: List[int], num_partitions: int,
                      world: Optional[World] = None):
    """Collective: this rank's share of the partitions of `table` as
    (full_name, full_shape, extents, tensor) slices for `write_bundle`.
    Partition k goes to rank k % W."""
    W = table.W
    out = []
    for k, (lo, n) in enumerate(partition_extents(table.num_rows, num_partitions)):
        t = gather_rows(table, lo, lo + n, k % W)
        if t is not None:
            ext = [(lo, n)] + [(0, int(d)) for d in full_shape[1:]]
            out.append((name, list(full_shape), ext, t.reshape([n] + list(full_shape[1:]))))
    return out


def restore_table(prefix: str, name: str, table: ShardedEmbedding, entry: Optional[dict] = None) -> None:
    """Load the rows this rank owns from a sliced (any partitioning along
    axis 0) or plain full entry."""
    e = entry or read_bundle_index(prefix)[name]
    rows, dim = table.num_rows, table.dim
    shape = list(e["shape"])
    if shape[0] != rows or (1 if len(shape) == 1 else shape[1]) != dim:
        raise ValueError(f"shape mismatch for {name}: ckpt {shape} vs table [{rows}, {dim}]")
    if not e["has_slices"]:
        table.load_full(read_tensor(prefix, name).reshape(rows, dim).float())
        return
    W, r = table.W, table.rank
    covered = 0
    with torch.no_grad():
        for ext, t in iter_slices(prefix, name, e):
            lo, n = ext[0]
            if n < 0:
                lo, n = 0, rows
            if any(b >= 0 and (a != 0 or b != dim) for a, b in ext[1:]):
                raise ValueError(f"{name}: only row-partitioned slices can be restored into a sharded table")
            i0, i1 = _owned(r, W, lo, lo + n)
            if i1 > i0:
                first = r + i0 * W - lo
                table.local[i0:i1].copy_(t.reshape(n, dim)[first:first + (i1 - i0) * W:W].to(table.device, torch.float32))
            covered += n
    if covered != rows:
        raise ValueError(f"slices of {name} in {prefix} cover {covered} of {rows} rows")


def save_sharded(prefix: str, local: Dict[str, Union[torch.Tensor, ShardedEmbedding]],
                 replicated: Optional[Dict[str, torch.Tensor]] = None, world: Optional[World] = None,
                 global_step: Optional[int] = None, num_partitions: Union[int, Dict[str, int], None] = None) -> str:
    """Collective save.  `local`: {full_name: ShardedEmbedding} tables, saved as
    TF partitioned variables with `num_partitions` partitions (default: one per
    rank); plain tensors in `local` are per-rank entries written by their rank.
    `replicated` tensors are written once by the chief."""
    w = world or get_world()
    if global_step is not None:
        prefix = f"{prefix}-{int(global_step)}"
    tensors, slices = {}, []
    for name in sorted(local):
        v = local[name]
        if isinstance(v, ShardedEmbedding):
            P = num_partitions.get(name, w.world_size) if isinstance(num_partitions, dict) else \
                (num_partitions or w.world_size)
            slices += gather_partitions(v, name, [v.num_rows, v.dim], P, w)
        else:
            tensors[name] = v
    if w.rank == 0 and replicated:
        tensors.update(replicated)
    if w.world_size == 1:
        write_bundle(prefix, tensors, slices=slices)
    else:
        write_bundle(prefix, tensors, shard_id=w.rank, num_shards=w.world_size, slices=slices)
        w.barrier()
        if w.rank == 0:
            _native.load().bundle_merge_shard_indexes(prefix, w.world_size, True)
    if w.rank == 0:
        d = os.path.dirname(os.path.abspath(prefix))
        update_checkpoint_state(d, os.path.abspath(prefix))
    w.barrier()
    return prefix


def restore_sharded(prefix: str, names: Dict[str, Union[torch.Tensor, ShardedEmbedding]]) -> None:
    """Copy checkpoint tensors into the given destinations (by name); tables
    take the rows they own."""
    idx = read_bundle_index(prefix)
    for name, dst in names.items():
        if name not in idx:
            raise KeyError(f"{name} not in checkpoint {prefix}")
        if isinstance(dst, ShardedEmbedding):
            restore_table(prefix, name, dst, idx[name])
            continue
        t = read_tensor(prefix, name)
        if tuple(t.shape) != tuple(dst.shape):
            raise ValueError(f"shape mismatch for {name}: {tuple(t.shape)} vs {tuple(dst.shape)}")
        with torch.no_grad():
            dst.copy_(t.to(dst.device, dst.dtype))
