"""Max pooling on channels_last bf16 activations (csrc/kernels/pool.hip):
forward stores each output's window position as one byte, backward gathers
(no atomics).  Any other case (CPU, fp32, NCHW, dilation, ceil_mode) is
`F.max_pool2d`."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import _native


class _MaxPoolNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        N, C, H, W = x.shape
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        y = torch.empty((N, C, Ho, Wo), device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
        idx = torch.empty(y.numel(), device=x.device, dtype=torch.uint8)
        _native.load().maxpool_fwd(x, y, idx, k, s, p)
        ctx.save_for_backward(idx)
        ctx.conf = (x.shape, k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        shape, k, s, p = ctx.conf
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = torch.empty(shape, device=dy.device, dtype=dy.dtype, memory_format=torch.channels_last)
        _native.load().maxpool_bwd(dy, idx, dx, k, s, p)
        return dx, None, None, None


def max_pool2d(x: torch.Tensor, kernel_size: int, stride: int, padding: int = 0) -> torch.Tensor:
    if (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last) and 2 * padding <= kernel_size
            and kernel_size * kernel_size <= 255):
        return _MaxPoolNHWC.apply(x, int(kernel_size), int(stride), int(padding))
    return F.max_pool2d(x, kernel_size, stride, padding)
