"""gemm_big tiling experiments on the forward layout: (BM, BK, stages) configs
vs hipBLASLt, interleaved rounds, random data, median TFLOP/s."""
import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
from distributed_tensorflow_example_amd import _native  # noqa: E402

CFG = {0: "256x256 BK32 S5", 1: "256x256 BK64 S2", 2: "128x256 BK64 S3", 3: "128x256 BK32 S5",
       4: "256x256 BK32 S3", 5: "128x256 BK64 S2", 6: "256x256 BK64 S2 reads-first+setprio",
       7: "256x256 BK64 S2 setprio", 8: "256x256 BK64 register-staged",
       9: "256x256 BK64 S2 one barrier per tile"}
C = _native.load()
for (M, N, K) in [(16384, 3072, 768), (16384, 768, 3072), (8192, 8192, 8192)]:
    torch.cuda.empty_cache()
    a = torch.randn(M, K, device="cuda").bfloat16()
    b = torch.randn(N, K, device="cuda").bfloat16()
    o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ref = (a.float() @ b.float().t())
    fns = {name: (lambda c=c: C.gemm_big_cfg(c, a, b, o)) for c, name in CFG.items()}
    fns["hipblaslt"] = lambda: torch.mm(a, b.t(), out=o)
    for name, f in fns.items():
        f()
        torch.cuda.synchronize()
        err = float((o.float() - ref).norm() / ref.norm())
        assert err < 1e-2, (name, err)
    t = {k: [] for k in fns}
    for _ in range(5):
        for k, f in fns.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                f()
            e.record()
            e.synchronize()
            t[k].append(s.elapsed_time(e) / 10)
    print(json.dumps({"M": M, "N": N, "K": K, **{k: round(2.0 * M * N * K / statistics.median(v) / 1e9, 1)
                                                  for k, v in t.items()}}), flush=True)
