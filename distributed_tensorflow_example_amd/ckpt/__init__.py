"""Distributed TF-format checkpoints: every rank writes its own data shard.

A TF V2 bundle may span N data files (`prefix.data-0000k-of-0000N`) with one
merged `prefix.index`.  Sharded state (row-sharded embedding tables, the
parameter-server part of the model) is written by its owning rank in
parallel -- no gather of a 1e9-row table onto one host -- and the chief
merges the per-shard index tables (native `bundle_merge_shard_indexes`) and
updates the `checkpoint` state file.  Replicated tensors are written once,
by the chief, into shard 0.  Names follow TF's partitioned variables:
`weights/Variable/part_3`.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import torch

from .. import _native
from ..compat.saver import latest_checkpoint, read_bundle_index, read_tensor, update_checkpoint_state, write_bundle
from ..parallel.world import World, get_world

__all__ = ["save_sharded", "restore_sharded", "latest_checkpoint", "read_tensor", "read_bundle_index"]


def save_sharded(prefix: str, local: Dict[str, torch.Tensor], replicated: Optional[Dict[str, torch.Tensor]] = None,
                 world: Optional[World] = None, global_step: Optional[int] = None) -> str:
    w = world or get_world()
    if global_step is not None:
        prefix = f"{prefix}-{int(global_step)}"
    tensors = dict(local)
    if w.rank == 0 and replicated:
        tensors.update(replicated)
    if w.world_size == 1:
        write_bundle(prefix, tensors)
    else:
        write_bundle(prefix, tensors, shard_id=w.rank, num_shards=w.world_size)
        w.barrier()
        if w.rank == 0:
            _native.load().bundle_merge_shard_indexes(prefix, w.world_size, True)
    if w.rank == 0:
        d = os.path.dirname(os.path.abspath(prefix))
        update_checkpoint_state(d, os.path.abspath(prefix))
    w.barrier()
    return prefix


def restore_sharded(prefix: str, names: Dict[str, torch.Tensor]) -> None:
    """Copy checkpoint tensors into the given destination tensors (by name)."""
    idx = read_bundle_index(prefix)
    for name, dst in names.items():
        if name not in idx:
            raise KeyError(f"{name} not in checkpoint {prefix}")
        t = read_tensor(prefix, name)
        if tuple(t.shape) != tuple(dst.shape):
            raise ValueError(f"shape mismatch for {name}: {tuple(t.shape)} vs {tuple(dst.shape)}")
        with torch.no_grad():
            dst.copy_(t.to(dst.device, dst.dtype))
