"""BERT-base weight-gradient paths at T = 16384 tokens (B=128, S=128), fp32
accumulate into an existing grad (beta = 1), us per call:
  addmm     one hipBLASLt GEMM, out_dtype fp32, beta = 1 (no extra pass)
  slabs     models/bert.py _wgrad_torch: token-slab bmm + slab_sum (the default fallback)
  gemm_big  in-tree 8-phase GEMM, split-K slabs + slab_reduce
One JSON line per shape."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_tensorflow_example_amd.models.bert import _wgrad_torch  # noqa: E402
from distributed_tensorflow_example_amd.ops import big_gemm  # noqa: E402


def timeit(fn, it=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e6


T = 16384
for out, inp in [(2304, 768), (768, 768), (3072, 768), (768, 3072)]:
    gy = torch.randn(T, out, device="cuda").bfloat16()
    x = torch.randn(T, inp, device="cuda").bfloat16()
    g = torch.zeros(out, inp, device="cuda")
    res = {"out": out, "in": inp}
    res["addmm_us"] = round(timeit(lambda: torch.addmm(g, gy.t(), x, out_dtype=torch.float32, out=g)), 1)
    res["slabs_us"] = round(timeit(lambda: _wgrad_torch(gy, x, into=g)), 1)
    res["gemm_big_us"] = round(timeit(lambda: big_gemm.linear_dw(gy, x, into=g)), 1)
    print(json.dumps(res), flush=True)
