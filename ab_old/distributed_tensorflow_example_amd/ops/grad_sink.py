"""Gradient sinks: backward kernels that accumulate a weight gradient straight
into the parameter's `.grad` (the DDP bucket view) instead of returning it.

Autograd's normal route for a bf16-compute / fp32-master weight is three device
passes per parameter per step -- the op's bf16 gradient, a bf16->fp32 cast
(autocast's ToCopyBackward), and AccumulateGrad's add into `.grad`.  A sunk
gradient is produced once, already accumulated: the fused BN backward adds
dgamma/dbeta in its finalize kernel, the conv backward does one mixed-dtype
`add_`, the BERT GEMMs run hipBLASLt with beta = 1 onto `.grad`.

Sinking is opt-in per parameter: `parallel.ddp.DistributedDataParallel`
installs `_dtf_sink_hook` (its bucket-ready callback) on every parameter it
manages; ops only sink into parameters that carry it, and call the hook
afterwards exactly where AccumulateGrad would have fired the
post-accumulate-grad hook.  Without the attribute gradients flow through
autograd as usual (so `torch.autograd.grad` and plain training keep their
semantics).
"""
from __future__ import annotations

import torch

_HOOK = "_dtf_sink_hook"


def enabled(p: torch.Tensor) -> bool:
    # a tied parameter (used by several ops, e.g. BERT's word embedding and
    # decoder) must reach .grad through autograd, which sums its uses and fires
    # the bucket-ready hook once
    return getattr(p, _HOOK, None) is not None and p.requires_grad and not getattr(p, "_dtf_tied", False)


def all_enabled(*params) -> bool:
    """Every given parameter sinks (and any existing .grad is a plain contiguous
    fp32 buffer the kernels can accumulate into)."""
    for p in params:
        if p is None or not enabled(p) or p.dtype != torch.float32:
            return False
        if p.grad is not None and not p.grad.is_contiguous():
            return False
    return True


def mark_tied(p: torch.Tensor) -> None:
    p._dtf_tied = True


def target(p: torch.Tensor) -> torch.Tensor:
    """The tensor to accumulate p's gradient into (created zeroed if absent)."""
    g = p.grad
    if g is None:
        g = torch.zeros_like(p, memory_format=torch.preserve_format)
        p.grad = g
    return g


def done(p: torch.Tensor) -> None:
    hook = getattr(p, _HOOK, None)
    if hook is not None:
        hook(p)


def install(p: torch.Tensor, hook) -> None:
    setattr(p, _HOOK, hook)


def uninstall(p: torch.Tensor) -> None:
    if hasattr(p, _HOOK):
        delattr(p, _HOOK)
