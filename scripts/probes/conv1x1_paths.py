"""ResNet-50 (B=128) 1x1 / stride-1 convolutions as GEMMs over the NHWC rows:
MIOpen (F.conv2d / its input gradient) vs hipBLASLt (torch.mm) vs the in-tree
gemm_big, us per call for the forward y = x W^T and the input gradient dx = dy W.
One JSON line per shape."""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_tensorflow_example_amd import _native  # noqa: E402

torch.backends.cudnn.benchmark = True


def timeit(fn, it=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e6


C = _native.load()
N = 128
# (cin, cout, hw) of the 1x1 stride-1 convs: stage 1..4 conv1 / conv3 (+ stage 1's downsample)
shapes = [(64, 64, 56), (64, 256, 56), (256, 64, 56), (256, 128, 56), (128, 512, 28), (512, 128, 28),
          (512, 256, 28), (256, 1024, 14), (1024, 256, 14), (1024, 512, 14), (512, 2048, 7), (2048, 512, 7)]
for cin, cout, hw in shapes:
    x = torch.randn(N, cin, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, 1, 1, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, cout, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
    dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)
    w2 = w.view(cout, cin)
    y2 = torch.empty(x2.shape[0], cout, device="cuda", dtype=torch.bfloat16)
    dx2 = torch.empty(x2.shape[0], cin, device="cuda", dtype=torch.bfloat16)
    r = {"cin": cin, "cout": cout, "hw": hw}
    r["fwd_miopen"] = round(timeit(lambda: F.conv2d(x, w)), 1)
    r["fwd_hipblaslt"] = round(timeit(lambda: torch.mm(x2, w2.t(), out=y2)), 1)
    r["fwd_gemm_big"] = round(timeit(lambda: C.gemm_big(x2, False, w2, True, y2)), 1)
    r["dx_miopen"] = round(timeit(lambda: torch.ops.aten.convolution_backward(
        dy, x, w, None, (1, 1), (0, 0), (1, 1), False, [0, 0], 1, [True, False, False])), 1)
    r["dx_hipblaslt"] = round(timeit(lambda: torch.mm(dy2, w2, out=dx2)), 1)
    r["dx_gemm_big"] = round(timeit(lambda: C.gemm_big(dy2, False, w2, False, dx2)), 1)
    print(json.dumps(r), flush=True)
