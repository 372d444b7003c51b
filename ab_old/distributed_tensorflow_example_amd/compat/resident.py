"""Resident Session engines: kernels that stay launched across Session.run calls.

The reference's hot loop is `sess.run([train_op, cost, summary_op,
global_step], feed_dict={x, y_})` every step (example.py:164-171).  On one
GPU the lowered MLP step (compat/lowering.py) can keep the persistent fp32
kernel resident instead of launching per run (csrc/bind_mlp.cpp
ResidentMLPPlan, csrc/kernels/mlp_persist_f32.hip RES): the host writes the
batch into pinned memory and rings a doorbell, the kernel trains one step on
the graph's own variables and writes loss / accuracy / global_step back.

A resident kernel holds the weights in registers, so anything else that
WRITES the graph's variables must stop it first: every Session.run that does
not take the resident path, `Variable.load`, `Saver.restore` and
`Session.close` call `quiesce_all()` (the kernel writes the variables through
every step, so reads need nothing).  A launch also exits by itself after
`DTF_RESIDENT_IDLE_S` (default 2 ms) without a run -- the next run relaunches
it (~20 us) -- and at interpreter exit.  The idle bound is short on purpose: a
device-wide `torch.cuda.synchronize()` waits for the resident launch too, so
it returns at most that long after the last run.  Direct torch writes to a variable's tensor
while an engine is live are not seen by it (call `quiesce_all()` first).
DTF_RESIDENT_SESSION=0 disables the engine.
"""
from __future__ import annotations

import atexit
import os

_LIVE: list = []     # handles whose launch may be live (a plain list: its truth test is free per run)


def enabled() -> bool:
    return os.environ.get("DTF_RESIDENT_SESSION", "1") != "0"


def idle_s() -> float:
    return float(os.environ.get("DTF_RESIDENT_IDLE_S", "0.002"))


class ResidentHandle:
    """Python owner of one native ResidentMLPPlan (registered while live)."""

    def __init__(self, native_plan):
        self.plan = native_plan
        self.out = native_plan.host_metrics().numpy()     # pinned [loss, accuracy, global_step]
        self.live = False

    def run_u8(self, u8, y, lr) -> bool:
        ok = self.plan.run_u8(u8, y, lr)
        if ok and not self.live:
            self.live = True
            _LIVE.append(self)
        return ok

    def stop(self):
        if self.live:
            self.live = False
            _LIVE.remove(self)
        self.plan.stop()


def any_live() -> bool:
    return bool(_LIVE)


def quiesce_all():
    """Stop every live resident engine (the variables already hold their values)."""
    if not _LIVE:
        return
    for h in list(_LIVE):
        h.stop()


atexit.register(quiesce_all)
