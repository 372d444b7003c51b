"""ResNet-50 (B=128) weight gradients on the in-tree implicit GEMM
(csrc/kernels/conv_igemm.hip conv_wgrad + wgrad_reduce) for the split plan
set by DTF_CONV_WGRAD_WGS / DTF_CONV_WGRAD_MINSTEPS (read once per process:
run once per setting), with MIOpen's weight gradient + the fp32 add for
reference.  us per call; one JSON line per shape.

    DTF_CONV_WGRAD_WGS=1024 python scripts/probes/conv_wgrad_sweep.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from distributed_tensorflow_example_amd.ops import big_gemm, conv

    B = 128
    cl = torch.channels_last
    shapes = [(1, 64, 256, 56, 1), (1, 256, 64, 56, 1), (1, 64, 64, 56, 1), (1, 256, 128, 56, 1),
              (1, 128, 512, 28, 1), (1, 512, 128, 28, 1), (1, 256, 1024, 14, 1), (1, 1024, 256, 14, 1),
              (1, 512, 2048, 7, 1), (1, 2048, 512, 7, 1),
              (3, 64, 64, 56, 1), (3, 128, 128, 56, 2), (3, 128, 128, 28, 1), (3, 256, 256, 28, 2),
              (3, 256, 256, 14, 1), (3, 512, 512, 14, 2), (3, 512, 512, 7, 1)]
    tag = {"wgs": os.environ.get("DTF_CONV_WGRAD_WGS", "512"), "depth": os.environ.get("DTF_CONV_WGRAD_DEPTH", "3"),
           "minsteps": os.environ.get("DTF_CONV_WGRAD_MINSTEPS", "8")}
    for ks, C, K, H, s in shapes:
        x = torch.randn(B, C, H, H, device="cuda").bfloat16().contiguous(memory_format=cl)
        Ho = (H - 1) // s + 1
        dy = torch.randn(B, K, Ho, Ho, device="cuda").bfloat16().contiguous(memory_format=cl)
        acc = torch.zeros((K, C, ks, ks), device="cuda").contiguous(memory_format=cl)
        r = dict(tag, ks=ks, C=C, K=K, H=H, stride=s)
        r["igemm_us"] = round(big_gemm._time(lambda: conv.conv3x3_dw(dy, x, s, into=acc), reps=10) * 1e3, 1)
        if os.environ.get("DTF_CONV_WGRAD_WGS") is None:
            w = torch.empty((K, C, ks, ks), device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)

            def miopen():
                dw = torch.ops.aten.convolution_backward(dy, x, w, None, (s, s), (ks // 2, ks // 2), (1, 1), False,
                                                         [0, 0], 1, [False, True, False])[1]
                acc.add_(dw)
            r["miopen_us"] = round(big_gemm._time(miopen, reps=10) * 1e3, 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
