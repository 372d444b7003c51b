"""Cost of a weight-gradient sink add (fp32 .grad += MIOpen's bf16 dW) per
layout of the two operands, and the strides MIOpen returns for a
channels_last weight: the ResNet-50 trace shows 50-70 us adds for 9-37K
element filters (profiles/resnet50_sink_add_r5.txt)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from distributed_tensorflow_example_amd.ops import big_gemm

    cl = torch.channels_last
    for (C, K, H, ks, s) in ((64, 64, 56, 3, 1), (3, 64, 224, 7, 2)):
        x = torch.randn(128, C, H, H, device="cuda").bfloat16().contiguous(memory_format=cl)
        Ho = (H + 2 * (ks // 2) - ks) // s + 1
        dy = torch.randn(128, K, Ho, Ho, device="cuda").bfloat16().contiguous(memory_format=cl)
        w = torch.randn(K, C, ks, ks, device="cuda").bfloat16().contiguous(memory_format=cl)
        dw = torch.ops.aten.convolution_backward(dy, x, w, None, (s, s), (ks // 2, ks // 2), (1, 1), False, [0, 0], 1,
                                                 [False, True, False])[1]
        r = {"shape": [K, C, ks, ks], "dw_stride": list(dw.stride()), "dw_dtype": str(dw.dtype)}
        for name, fmt in (("cl", cl), ("contig", torch.contiguous_format)):
            g = torch.zeros(K, C, ks, ks, device="cuda").contiguous(memory_format=fmt)
            r[f"add_into_{name}_us"] = round(big_gemm._time(lambda: g.add_(dw), reps=20) * 1e3, 2)
            dwf = dw.contiguous(memory_format=fmt)
            r[f"add_into_{name}_matched_us"] = round(big_gemm._time(lambda: g.add_(dwf), reps=20) * 1e3, 2)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
