"""Race / consistency checks and fault injection.

The reference has neither: Hogwild updates race by design and every lr2.py
worker re-runs init_op (a race by accident).  Synchronous DP removes both;
what remains worth checking is that replicas stay bit-identical, and the
failure paths need a way to be exercised:

* `replica_checksum(tensors)` / `assert_replicas_consistent(world, tensors)` --
  fp64 sum + abs-sum + a position-weighted sum, compared across ranks
  (max == min); `DTF_CHECK_REPLICAS_EVERY=N` turns it on inside the compat
  train op every N steps;
* `fault_point(step)` -- `DTF_FAULT_STEP=k [DTF_FAULT_RANK=r]
  [DTF_FAULT_MODE=raise|exit|abort]` makes rank r fail at step k (tests of
  the launcher teardown and checkpoint restart);
* `serialize_kernels()` -- AMD_SERIALIZE_KERNEL=3 / HIP_LAUNCH_BLOCKING style
  debugging for the GPU path (must be set before the HIP runtime starts).
"""
from __future__ import annotations

import os
import sys
from typing import Iterable

import torch


class InjectedFault(RuntimeError):
    pass


def fault_point(step: int, rank: int = None):
    k = os.environ.get("DTF_FAULT_STEP")
    if k is None or int(k) != int(step):
        return
    want = os.environ.get("DTF_FAULT_RANK")
    if rank is None:
        rank = int(os.environ.get("RANK", os.environ.get("DTF_TASK_RANK", 0)))
    if want is not None and int(want) != int(rank):
        return
    mode = os.environ.get("DTF_FAULT_MODE", "raise")
    msg = f"injected fault at step {step} on rank {rank}"
    if mode == "exit":
        sys.stderr.write(msg + "\n")
        sys.stderr.flush()
        os._exit(17)
    if mode == "abort":
        os.abort()
    raise InjectedFault(msg)


def replica_checksum(tensors: Iterable[torch.Tensor]) -> torch.Tensor:
    s = torch.zeros(3, dtype=torch.float64)
    for t in tensors:
        v = t.detach().reshape(-1).double().cpu()
        w = torch.arange(1, v.numel() + 1, dtype=torch.float64) / max(1, v.numel())
        s += torch.stack([v.sum(), v.abs().sum(), (v * w).sum()])
    return s


def assert_replicas_consistent(world, tensors: Iterable[torch.Tensor], what: str = "params"):
    if world is None or world.world_size <= 1:
        return True
    c = replica_checksum(list(tensors))
    for i in range(3):
        hi = world.host_all_reduce(float(c[i]), "max")
        lo = world.host_all_reduce(float(c[i]), "min")
        if hi != lo:
            raise AssertionError(f"replicas diverged ({what}): checksum[{i}] spread {hi - lo}")
    return True


def check_every() -> int:
    return int(os.environ.get("DTF_CHECK_REPLICAS_EVERY", "0"))


def serialize_kernels():
    os.environ.setdefault("AMD_SERIALIZE_KERNEL", "3")
    os.environ.setdefault("HIP_LAUNCH_BLOCKING", "1")
