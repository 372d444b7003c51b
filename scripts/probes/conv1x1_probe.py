"""Probe: ResNet-50 1x1 convs through MIOpen (immediate vs find) vs hipBLASLt GEMMs.

fwd + bwd-data + wgrad for NHWC bf16 tensors; the GEMM path produces the
weight gradient in fp32 directly (torch.mm out_dtype), as the master weights are fp32.
"""
import time

import torch
import torch.nn.functional as F


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.time()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.time() - t) / it * 1e6


SHAPES = [(128, 56, 64, 256), (128, 56, 256, 64), (128, 28, 512, 128), (128, 28, 128, 512),
          (128, 14, 1024, 256), (128, 14, 256, 1024), (128, 7, 2048, 512), (128, 7, 512, 2048)]
for bench in (False, True):
    torch.backends.cudnn.benchmark = bench
    tot_c = tot_g = 0.0
    for N, HW, cin, cout in SHAPES:
        x = torch.randn(N, cin, HW, HW, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, 1, 1, device="cuda") * 0.05).bfloat16()
        dy = torch.randn(N, cout, HW, HW, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        xr = x.detach().requires_grad_()
        wr = w.detach().requires_grad_()

        def conv():
            y = F.conv2d(xr, wr)
            y.backward(dy)

        x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
        dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)
        w2 = w.view(cout, cin)

        def gemm():
            torch.mm(x2, w2.t())
            torch.mm(dy2, w2)
            torch.mm(dy2.t(), x2, out_dtype=torch.float32)

        tc, tg = timeit(conv), timeit(gemm)
        tot_c += tc
        tot_g += tg
        print(f"find={int(bench)} N{N} HW{HW} {cin}->{cout}: miopen {tc:8.1f} us  gemm {tg:8.1f} us", flush=True)
    print(f"find={int(bench)} total miopen {tot_c:.1f} us gemm {tot_g:.1f} us", flush=True)
