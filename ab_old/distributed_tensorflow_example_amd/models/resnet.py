"""ResNet-50 (v1.5) on synthetic ImageNet-shaped input (BASELINE config #3).

Not in the reference.  MI355X layout: channels_last (NHWC)
bf16 activations so MIOpen picks its implicit-GEMM MFMA convolutions, fp32
master weights updated by the fused multi-tensor momentum kernel, the loss
by the fused softmax-xent kernel, and gradients averaged by the bucketed
DDP all-reduce overlapped with backward (parallel.ddp).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..ops.bn import FusedBatchNorm2d
from ..ops.conv import ShadowConv2d, XGradShare, attach_shadows as _attach_conv_shadows
from ..ops.pool import max_pool2d
from ..ops.transformer import GradSlot


class Bottleneck(nn.Module):
    expansion = 4
    # identity blocks: conv1's dx GEMM accumulates the residual gradient (DTF_RES_FOLD=0: autograd adds)
    fold_residual_grad = os.environ.get("DTF_RES_FOLD", "1") != "0"
    # downsampling blocks: conv1 / projection input gradients folded into one tensor (DTF_X_SHARE=0: autograd adds)
    share_input_grad = os.environ.get("DTF_X_SHARE", "1") != "0"

    def __init__(self, cin, width, stride=1, down=False):
        super().__init__()
        cout = width * 4
        self.conv1 = ShadowConv2d(cin, width, 1, bias=False)
        self.bn1 = FusedBatchNorm2d(width)
        self.conv2 = ShadowConv2d(width, width, 3, stride, 1, bias=False)   # v1.5: stride on the 3x3
        self.bn2 = FusedBatchNorm2d(width)
        self.conv3 = ShadowConv2d(width, cout, 1, bias=False)
        self.bn3 = FusedBatchNorm2d(cout)
        nn.init.zeros_(self.bn3.weight)                                  # zero-init last BN gamma
        self.down_conv = ShadowConv2d(cin, cout, 1, stride, bias=False) if down else None
        self.down_bn = FusedBatchNorm2d(cout) if down else None

    def _fold_ok(self, x) -> bool:
        """The fold needs conv1 on its bf16-shadow path, the only one that takes the
        slot: a gradient bn3 deposited for any other path would be lost.  (A bn3
        off its fused path ignores the slot and returns the gradient itself.)"""
        return (self.fold_residual_grad and self.down_conv is None and self.training
                and self.conv1.on_shadow_path(x))

    def _share_ok(self, x) -> bool:
        """Downsampling blocks: conv1 and the projection both read x and both take
        the shared input-gradient fold (each must be on its shadow path)."""
        return (self.share_input_grad and self.down_conv is not None and self.training and x.requires_grad
                and self.conv1.on_shadow_path(x) and self.down_conv.on_shadow_path(x))

    def forward(self, x):
        # downsampling blocks: the projection's and conv1's input gradients meet
        # in one tensor (GEMM beta = 1, or the stride-2 projection's strided
        # pixels added in place) instead of MIOpen's zero-filled dx + an add
        share = XGradShare() if self._share_ok(x) else None
        idt = self.down_bn(self.down_conv(x, share=share)) if self.down_conv is not None else x
        # identity path: bn3's residual gradient is accumulated by conv1's input-
        # gradient GEMM (beta = 1) instead of autograd adding the two branches
        slot = GradSlot() if self._fold_ok(x) else None
        y = self.bn1(self.conv1(x, grad_slot=slot, share=share), relu=True)   # BN + ReLU: one fused pass
        y = self.bn2(self.conv2(y), relu=True)
        return self.bn3(self.conv3(y), residual=idt, relu=True, residual_slot=slot)   # BN + residual add + ReLU


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes=1000):
        super().__init__()
        self.conv1 = ShadowConv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = FusedBatchNorm2d(64)
        blocks, cin = [], 64
        for i, (n, w) in enumerate(zip(layers, (64, 128, 256, 512))):
            for j in range(n):
                blocks.append(Bottleneck(cin, w, stride=(2 if (i > 0 and j == 0) else 1), down=(j == 0)))
                cin = w * 4
        self.blocks = nn.Sequential(*blocks)
        self.fc = nn.Linear(cin, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def forward(self, x):
        with torch.autocast(device_type="cuda", dtype=torch.bfloat16, enabled=x.is_cuda):
            x = self.bn1(self.conv1(x), relu=True)
            x = max_pool2d(x, 3, 2, 1)
            x = self.blocks(x)
            x = torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
            return self.fc(x)

    def attach_shadows(self, optimizer=None):
        """bf16 conv weights maintained by the fused optimizer (ops.conv)."""
        _attach_conv_shadows(self, optimizer)

    def loss(self, images, labels):
        return ops.softmax_xent(self.forward(images).float(), labels)


def resnet50(num_classes: int = 1000) -> ResNet:
    return ResNet((3, 4, 6, 3), num_classes)


def synthetic_imagenet_batch(batch: int, device, seed: int = 0, size: int = 224, num_classes: int = 1000):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(batch, 3, size, size, generator=g).to(device).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, num_classes, (batch,), generator=g).to(device)
    return x, y
