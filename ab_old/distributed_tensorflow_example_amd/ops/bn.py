"""Fused BatchNorm2d (+residual add)(+ReLU) on NHWC bf16 (csrc/kernels/bn.hip).

`FusedBatchNorm2d` is a drop-in nn.BatchNorm2d whose forward takes an
optional residual and a relu flag: in training on a channels_last bf16 GPU
activation it runs the fused kernels (stats, normalise+affine+add+ReLU in one
pass; backward recomputes x_hat and the ReLU mask from x); otherwise it runs
the equivalent PyTorch ops (CPU oracle / eval / other layouts).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn.functional as F

from .. import _native
from . import grad_sink


def _C():
    return _native.load()


def _nhwc(x: torch.Tensor) -> bool:
    return x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)


# DTF_FUSED_BN=0 routes every layer through MIOpen's BN + separate add/ReLU (A/B runs)
_ENABLED = os.environ.get("DTF_FUSED_BN", "1") != "0"
# DTF_BN_BWD_EPILOGUE=0: no BN-backward partials from the consuming convolution's
# input-gradient epilogue (A/B runs)
_BWD_EPI = os.environ.get("DTF_BN_BWD_EPILOGUE", "1") != "0"
_bwd_handoff = {}   # id(BN output) -> BwdSlot: from _FusedBN.forward to FusedBatchNorm2d.forward


class BwdSlot:
    """A BatchNorm (+ residual) + ReLU whose output's gradient may be produced
    by the consuming convolution's input-gradient kernel together with this BN's
    backward partials (ops/conv.py: the in-tree implicit GEMM's EPI 2 / 3
    epilogue masks the gradient with the ReLU and sums g and g * x_hat; with a
    residual the conv's gradient is first added onto the residual branch's).
    The conv's backward fills `part`, `g` and `g_version`; the BN's backward
    uses them when its incoming gradient is exactly that tensor, unmodified."""
    __slots__ = ("x", "stats", "res", "part", "g", "g_version")

    def __init__(self, x, stats, res=None):
        self.x, self.stats, self.res = x, stats, res
        self.part = self.g = self.g_version = None

    def take(self, dy):
        """(part, P) when dy is the conv's masked gradient, untouched since; else None."""
        part, g, ver = self.part, self.g, self.g_version
        self.part = self.g = self.g_version = None
        if part is None or g is None or dy.data_ptr() != g.data_ptr() or dy._version != ver or dy.shape != g.shape:
            return None
        return part


class _FusedBN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, res, running_mean, running_var, momentum, eps, relu, sink, res_slot=None,
                pre=None):
        C = _C()
        ch = gamma.numel()
        M = x.numel() // ch
        y = torch.empty_like(x)
        stats = torch.empty(4 * ch, dtype=torch.float32, device=x.device)
        if pre is not None:
            # x's producer (a 3x3 conv on the in-tree kernel) wrote the statistics partials
            part, P = pre
            C.bn_fwd_parts(x, res, gamma, beta, y, part, P, stats, running_mean, running_var, momentum, eps, relu)
        else:
            part = torch.empty(2 * C.bn_partial_rows(M, ch) * ch, dtype=torch.float32, device=x.device)
            C.bn_fwd(x, res, gamma, beta, y, part, stats, running_mean, running_var, momentum, eps, relu)
        ctx.save_for_backward(x, res if res is not None else torch.empty(0, device=x.device), gamma, stats)
        ctx.has_res, ctx.relu = res is not None, relu
        ctx.sink = sink           # (weight, bias) whose .grad the finalize kernel accumulates into, or None
        ctx.res_slot = res_slot   # GradSlot: the residual's gradient goes to the GEMM that consumes it
        ctx.bwd_slot = None
        if _BWD_EPI and relu:
            ctx.bwd_slot = BwdSlot(x, stats, res)
            _bwd_handoff[id(y)] = ctx.bwd_slot
        return y

    @staticmethod
    def backward(ctx, dy):
        C = _C()
        x, res, gamma, stats = ctx.saved_tensors
        ch = gamma.numel()
        M = x.numel() // ch
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = torch.empty_like(x)
        if ctx.sink is not None:
            dgamma, dbeta = grad_sink.target(ctx.sink[0]), grad_sink.target(ctx.sink[1])
        else:
            dgamma = torch.empty(ch, dtype=torch.float32, device=x.device)
            dbeta = torch.empty_like(dgamma)
        coef = torch.empty(3 * ch, dtype=torch.float32, device=x.device)
        pre = ctx.bwd_slot.take(dy) if ctx.bwd_slot is not None else None
        if pre is not None:
            # dy is already relu-masked and its partials came from the conv's epilogue;
            # the masked gradient is also the residual's gradient
            C.bn_bwd_parts(dy, x, gamma, stats, pre[0], pre[1], coef, dx, dgamma, dbeta, ctx.sink is not None)
            dres = dy if ctx.has_res else None
        else:
            dres = torch.empty_like(res) if ctx.has_res else None
            part = torch.empty(2 * C.bn_partial_rows(M, ch) * ch, dtype=torch.float32, device=x.device)
            C.bn_bwd(dy, x, res if ctx.has_res else None, gamma, stats, part, coef, dx, dres, dgamma, dbeta,
                     ctx.relu, ctx.sink is not None)
        if dres is not None and ctx.res_slot is not None and not ctx.res_slot.consumed:
            # folded into the residual source's other consumer: the 1x1 conv's dx GEMM
            # accumulates it (beta = 1) instead of autograd adding the two branches
            ctx.res_slot.g, dres = dres, None
        if ctx.sink is not None:
            grad_sink.done(ctx.sink[0])
            grad_sink.done(ctx.sink[1])
            return dx, None, None, dres, None, None, None, None, None, None, None, None
        return dx, dgamma, dbeta, dres, None, None, None, None, None, None, None, None


class FusedBatchNorm2d(torch.nn.BatchNorm2d):
    """BatchNorm2d whose training forward optionally fuses a residual add and ReLU.

    ``num_batches_tracked`` is only read by PyTorch when ``momentum is None``;
    on the fused path its increments are counted on the host and folded into
    the buffer when the state dict is taken, instead of one tiny device add per
    layer per step.
    """

    _pending_batches = 0

    def _flush_batches(self):
        if self._pending_batches and self.num_batches_tracked is not None:
            with torch.no_grad():
                self.num_batches_tracked += self._pending_batches
        self._pending_batches = 0

    def _sink(self):
        w, b = self.weight, self.bias
        ok = (grad_sink.enabled(w) and grad_sink.enabled(b)
              and all(p.grad is None or (p.grad.dtype == torch.float32 and p.grad.is_contiguous()) for p in (w, b)))
        return (w, b) if ok else None

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        self._flush_batches()
        super()._save_to_state_dict(destination, prefix, keep_vars)

    def forward(self, x, residual: Optional[torch.Tensor] = None, relu: bool = False,
                residual_slot=None):  # noqa: D401
        """`residual_slot` (ops.transformer.GradSlot, fused path only): the
        residual's gradient is handed to the slot's consumer instead of being
        returned through autograd."""
        fused_ok = (_ENABLED and self.training and x.is_cuda and x.dtype == torch.bfloat16 and _nhwc(x)
                    and self.affine and x.shape[1] % 8 == 0 and self.momentum is not None
                    and (residual is None or (residual.dtype == torch.bfloat16 and _nhwc(residual))))
        if fused_ok:
            if self.track_running_stats:
                self._pending_batches += 1
            mom = self.momentum
            pre = getattr(x, "_dtf_bn_part", None)
            if pre is not None:
                pre, ver = pre
                if ver != x._version or pre[0].dim() != 3 or pre[0].shape[2] != x.shape[1]:
                    pre = None          # y changed in place after the conv, or another layout
            y = _FusedBN.apply(x, self.weight, self.bias, residual, self.running_mean if self.track_running_stats
                               else None, self.running_var if self.track_running_stats else None, float(mom),
                               float(self.eps), bool(relu), self._sink(), residual_slot, pre)
            if _bwd_handoff:
                slot = _bwd_handoff.pop(id(y), None)
                _bwd_handoff.clear()
                if slot is not None:
                    y._dtf_bn_bwd = slot     # read by the ShadowConv2d that consumes y
            return y
        self._flush_batches()
        y = super().forward(x)
        if residual is not None:
            y = y + residual
        return F.relu(y) if relu else y
