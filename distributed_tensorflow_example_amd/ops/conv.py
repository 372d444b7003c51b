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
  no separate AccumulateGrad add;
* a 1x1 / stride-1 convolution's weight gradient is a plain GEMM over the
  NHWC rows, dW[cout, cin] = dy[NHW, cout]^T x[NHW, cin]: it can run on the
  in-tree GEMM (gemm_big.hip, split-K over the rows, fp32 out accumulated
  straight into the bucket) instead of MIOpen's atomic wrw solver, whose
  zero-fill + scale + fp32->bf16 cast passes and our bf16->fp32 add cost more
  than the GEMM itself (ResNet-50, profiles/resnet50_r4.md).  Both routes are
  timed once per shape (`DTF_CONV_GEMM_DW`: auto / never / always).
Any other case (CPU, no shadow, eval under a different dtype) is plain
`nn.Conv2d`.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import grad_sink

_DW_POLICY = os.environ.get("DTF_CONV_GEMM_DW", "auto")
_dw_choice: dict = {}
_dw_timings: dict = {}


def _gemm_dw_ok(x, dy, w16, stride, padding, dilation, groups) -> bool:
    return (w16.shape[2] == 1 and w16.shape[3] == 1 and tuple(stride) == (1, 1) and tuple(padding) == (0, 0)
            and groups == 1 and x.is_cuda and x.dtype == torch.bfloat16 and dy.dtype == torch.bfloat16
            and x.is_contiguous(memory_format=torch.channels_last)
            and dy.is_contiguous(memory_format=torch.channels_last)
            and (x.shape[0] * x.shape[2] * x.shape[3]) % 64 == 0)


def _rows(t):
    """[N, C, H, W] channels_last -> its [N*H*W, C] row view (no copy)."""
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])


def _use_gemm_dw(x, dy, w16) -> bool:
    """Per shape: the in-tree GEMM (accumulating into an fp32 target) vs MIOpen's
    weight gradient + the bf16 -> fp32 add, each timed once on these operands."""
    if _DW_POLICY == "never":
        return False
    if _DW_POLICY == "always":
        return True
    key = (tuple(x.shape), w16.shape[0])
    hit = _dw_choice.get(key)
    if hit is None:
        if torch.cuda.is_current_stream_capturing():
            return False
        from . import big_gemm
        acc = torch.zeros(w16.shape[0], w16.shape[1], device=x.device, dtype=torch.float32)
        x2, dy2 = _rows(x), _rows(dy)

        def ours():
            big_gemm.linear_dw(dy2, x2, into=acc)

        def miopen():
            dw = torch.ops.aten.convolution_backward(dy, x, w16, None, (1, 1), (0, 0), (1, 1), False, [0, 0], 1,
                                                     [False, True, False])[1]
            acc.add_(dw.view(acc.shape))
        t_ours, t_theirs = big_gemm._time(ours, reps=3), big_gemm._time(miopen, reps=3)
        hit = _dw_choice[key] = t_ours <= t_theirs
        _dw_timings[key] = (round(t_ours, 4), round(t_theirs, 4))
    return hit


def dw_choices() -> dict:
    """{(x shape, cout): (gemm chosen, (gemm ms, miopen ms))}"""
    return {k: (v, _dw_timings.get(k)) for k, v in _dw_choice.items()}


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
        w = ctx.w
        if need_w and _gemm_dw_ok(x, dy, w16, stride, padding, dilation, groups) and _use_gemm_dw(x, dy, w16):
            from . import big_gemm
            dx = (torch.ops.aten.convolution_backward(dy, x, w16, None, stride, padding, dilation, False, [0, 0],
                                                      groups, [True, False, False])[0] if need_x else None)
            sink = grad_sink.enabled(w) and (w.grad is None or w.grad.is_contiguous())
            if sink:
                g = grad_sink.target(w)
                big_gemm.linear_dw(_rows(dy), _rows(x), into=g.view(g.shape[0], g.shape[1]))
                grad_sink.done(w)
                return dx, None, None, None, None, None, None
            dw = big_gemm.linear_dw(_rows(dy), _rows(x)).view(w.shape)
            return dx, dw.to(w.dtype), None, None, None, None, None
        dx, dw, _ = torch.ops.aten.convolution_backward(dy, x, w16, None, stride, padding, dilation, False,
                                                        [0, 0], groups, [need_x, need_w, False])
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
