"""gemm_big: the same C[M,N] = A[M,K] B' product with B stored [N,K] (K-contiguous,
the forward's layout) vs [K,N] (N-contiguous, the input gradient's: read with
ds_read_b64_tr_b16), next to torch (hipBLASLt) on both, at BERT-base's shapes.
Usage: python scripts/probes/gemm_layout_ab.py [pmc <kc|nc> M N K]."""
import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
from distributed_tensorflow_example_amd import _native  # noqa: E402

C = _native.load()
bf = torch.bfloat16
dev = "cuda"


def timed(fn, reps=20, rounds=7):
    fn()
    ts = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) / reps)
    return statistics.median(ts)


def ops(M, N, K):
    a = torch.randn(M, K, device=dev, dtype=bf)
    bkc = torch.randn(N, K, device=dev, dtype=bf)          # [N, K]
    bnc = bkc.t().contiguous()                              # [K, N]
    o = torch.empty(M, N, device=dev, dtype=bf)
    return {"ours_kc": lambda: C.gemm_big(a, False, bkc, True, o),
            "ours_nc": lambda: C.gemm_big(a, False, bnc, False, o),
            "torch_kc": lambda: torch.mm(a, bkc.t(), out=o),
            "torch_nc": lambda: torch.mm(a, bnc, out=o)}


if len(sys.argv) > 1 and sys.argv[1] == "pmc":
    lay, M, N, K = sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    f = ops(M, N, K)["ours_" + lay]
    for _ in range(20):
        f()
    torch.cuda.synchronize()
    sys.exit(0)

for (M, N, K, what) in [(16384, 768, 3072, "ffn2 fwd / ffn1 dx"), (16384, 768, 2304, "qkv dx"),
                        (16384, 3072, 768, "ffn1 fwd / ffn2 dx"), (16384, 768, 768, "attn_out fwd / dx"),
                        (16384, 2304, 768, "qkv fwd")]:
    f = ops(M, N, K)
    r = {k: round(timed(v), 4) for k, v in f.items()}
    fl = 2.0 * M * N * K
    print(json.dumps({"M": M, "N": N, "K": K, "what": what, "ms": r,
                      "tflops": {k: round(fl / v / 1e9, 1) for k, v in r.items()}}), flush=True)
