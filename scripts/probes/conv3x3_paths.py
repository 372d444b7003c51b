"""ResNet-50 (B=128) 3x3 convolutions: in-tree implicit GEMM
(csrc/kernels/conv_igemm.hip) vs MIOpen -- forward, weight gradient (into an
fp32 buffer; MIOpen's bf16 result plus the add) and stride-1 input gradient,
us per call.  One JSON line per shape.

    python scripts/probes/conv3x3_paths.py [batch]
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from distributed_tensorflow_example_amd.ops import big_gemm, conv

    torch.backends.cudnn.benchmark = True
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    shapes = [(64, 56, 64, 1), (128, 56, 128, 2), (128, 28, 128, 1), (256, 28, 256, 2), (256, 14, 256, 1),
              (512, 14, 512, 2), (512, 7, 512, 1)]
    for C, H, K, s in shapes:
        x = torch.randn(B, C, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(K, C, 3, 3, device="cuda") * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
        Ho = (H - 1) // s + 1
        flop = 2.0 * B * Ho * Ho * K * C * 9
        r = {"C": C, "H": H, "K": K, "stride": s}
        r["fwd_miopen_us"] = round(big_gemm._time(lambda: F.conv2d(x, w, None, s, 1), reps=10) * 1e3, 1)
        r["fwd_igemm_us"] = round(big_gemm._time(lambda: conv.conv3x3(x, w, s), reps=10) * 1e3, 1)
        for bn in ((64, 128) if K % 128 == 0 else (64,)):
            r[f"fwd_igemm_bn{bn}_us"] = round(big_gemm._time(lambda: conv.conv3x3(x, w, s, bn=bn), reps=10) * 1e3, 1)
        P = conv.conv3x3_stat_rows(x, s)
        part = torch.empty(2, P, K, device="cuda")
        r["fwd_igemm_stats_us"] = round(big_gemm._time(lambda: conv.conv3x3(x, w, s, stats=part), reps=10) * 1e3, 1)
        r["fwd_igemm_tflops"] = round(flop / (r["fwd_igemm_us"] * 1e-6) / 1e12, 1)
        r["fwd_miopen_tflops"] = round(flop / (r["fwd_miopen_us"] * 1e-6) / 1e12, 1)
        dyo = torch.randn(B, K, Ho, Ho, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        acc = torch.zeros(K, C, 3, 3, device="cuda")
        r["dw_miopen_us"] = round(big_gemm._time(lambda: acc.add_(torch.ops.aten.convolution_backward(
            dyo, x, w, None, (s, s), (1, 1), (1, 1), False, [0, 0], 1, [False, True, False])[1]), reps=10) * 1e3, 1)
        r["dw_igemm_us"] = round(big_gemm._time(lambda: conv.conv3x3_dw(dyo, x, s, into=acc), reps=10) * 1e3, 1)
        if s == 1:
            dy = torch.randn(B, K, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
            r["dx_miopen_us"] = round(big_gemm._time(lambda: torch.ops.aten.convolution_backward(
                dy, x, w, None, (1, 1), (1, 1), (1, 1), False, [0, 0], 1, [True, False, False]), reps=10) * 1e3, 1)
            r["dx_igemm_us"] = round(big_gemm._time(lambda: conv.conv3x3_dx(dy, w, x.shape), reps=10) * 1e3, 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
