"""W&D tower GEMM shapes (B = 4096, 64-512-256-1, fp32): native gemm.hip vs torch, per shape."""
import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
from distributed_tensorflow_example_amd import _native  # noqa: E402

C = _native.load()
B = 4096
dims = [64, 512, 256, 1]
cases = []
for i in range(3):
    k, n = dims[i], dims[i + 1]
    cases.append(("fwd", B, n, k, False, False))        # X[B,k] W[k,n]
    cases.append(("dx", B, k, n, False, True))          # dZ[B,n] W[k,n]^T
    cases.append(("dw", k, n, B, True, False))          # X[B,k]^T dZ[B,n]
for role, M, N, K, tA, tB in cases:
    A = torch.randn(*((K, M) if tA else (M, K)), device="cuda")
    Bm = torch.randn(*((N, K) if tB else (K, N)), device="cuda")
    out = torch.empty(M, N, device="cuda")
    a_ = A.t() if tA else A
    b_ = Bm.t() if tB else Bm
    fns = {"native": lambda: C.gemm(A, tA, Bm, tB, out), "torch": lambda: torch.mm(a_, b_, out=out)}
    t = {k: [] for k in fns}
    for f in fns.values():
        f()
    for _ in range(5):
        for k, f in fns.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                f()
            e.record()
            e.synchronize()
            t[k].append(s.elapsed_time(e) / 20 * 1e3)
    print(json.dumps({"role": role, "M": M, "N": N, "K": K, **{k + "_us": round(statistics.median(v), 2)
                                                                for k, v in t.items()}}), flush=True)
