"""gemm_big weight-gradient split-K sweep on BERT-base dW shapes (T = 16384):
us per call of C.gemm_big(dy^T, x) accumulating into fp32 (beta = 1) for each
slab count (0 = the kernel's automatic choice).  One JSON line per shape."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_tensorflow_example_amd import _native  # noqa: E402


def timeit(fn, it=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e6


C = _native.load()
T = 16384
for out, inp in [(2304, 768), (768, 768), (3072, 768), (768, 3072)]:
    gy = torch.randn(T, out, device="cuda").bfloat16()
    x = torch.randn(T, inp, device="cuda").bfloat16()
    g = torch.zeros(out, inp, device="cuda")
    res = {"out": out, "in": inp}
    for sk in (0, 2, 4, 6, 8, 12, 16, 24, 32):
        res[f"split{sk}"] = round(timeit(lambda: C.gemm_big(gy, True, x, False, g, beta=1.0, split_k=sk)), 1)
    print(json.dumps(res), flush=True)
