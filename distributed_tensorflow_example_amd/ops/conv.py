"""Conv2d on the optimizer-maintained bf16 weight shadow, with a sunk wgrad.

The convolutions themselves stay on MIOpen (its implicit-GEMM MFMA solvers,
picked by solver search when `torch.backends.cudnn.benchmark` is on); what
this removes is the glue around them in a bf16-compute / fp32-master step:

* forward reads `weight._shadow` (bf16, same channels_last layout), which the
  fused optimizer rewrites in the same pass that updates the fp32 master --
  no per-step fp32->bf16 weight cast;
* backward asks MIOpen for (dx, dW) in one `convolution_backward` call and,
  when the weight is managed by DDP (ops.grad_sink), folds the bf16 dW into
  the fp32 bucket view with one mixed-dtype add -- no bf16->fp32 cast pass and
  no separate AccumulateGrad add.
Any other case (CPU, no shadow, eval under a different dtype) is plain
`nn.Conv2d`.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import grad_sink


class _ShadowConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, w16, stride, padding, dilation, groups):
        ctx.save_for_backward(x, w16)
        ctx.conf = (stride, padding, dilation, groups)
        ctx.w = w
        return F.conv2d(x, w16, None, stride, padding, dilation, groups)

    @staticmethod
    def backward(ctx, dy):
        x, w16 = ctx.saved_tensors
        stride, padding, dilation, groups = ctx.conf
        need_x = ctx.needs_input_grad[0]
        need_w = ctx.needs_input_grad[1]
        dy = dy.to(w16.dtype)
        dx, dw, _ = torch.ops.aten.convolution_backward(dy, x, w16, None, stride, padding, dilation, False,
                                                        [0, 0], groups, [need_x, need_w, False])
        w = ctx.w
        if need_w and grad_sink.enabled(w):
            grad_sink.target(w).add_(dw)
            grad_sink.done(w)
            return dx, None, None, None, None, None, None
        return dx, (dw.to(w.dtype) if need_w else None), None, None, None, None, None


class ShadowConv2d(torch.nn.Conv2d):
    """nn.Conv2d that computes with `weight._shadow` when one is attached."""

    def forward(self, x):
        w16 = getattr(self.weight, "_shadow", None)
        if (w16 is not None and x.is_cuda and self.bias is None and self.padding_mode == "zeros"
                and isinstance(self.padding, tuple)):
            if x.dtype != w16.dtype:
                x = x.to(w16.dtype)
            return _ShadowConv.apply(x, self.weight, w16, self.stride, self.padding, self.dilation, self.groups)
        return super().forward(x)


def attach_shadows(module: torch.nn.Module, optimizer=None, dtype=torch.bfloat16):
    """Give every ShadowConv2d weight a bf16 shadow kept current by `optimizer`
    (a fused optimizer's attach_shadow), or a one-off copy without one."""
    for m in module.modules():
        if isinstance(m, ShadowConv2d):
            w = m.weight
            if getattr(w, "_shadow", None) is None:
                w._shadow = torch.empty_like(w, dtype=dtype)
            if optimizer is not None:
                optimizer.attach_shadow(w, w._shadow)
            else:
                with torch.no_grad():
                    w._shadow.copy_(w)
