"""Time the BERT-base LayerNorm kernels in isolation at the B = 128, S = 128
shape ([16384, 768] bf16): bdrln_fwd (bias + dropout + residual + LN) and
ln_bwd (with the dropout-branch output and dgamma / dbeta / dbias partials).
Prints one JSON line: us per call and the HBM rate of the tensors each moves.
Run from a tree root (its own built extension): python scripts/probes/ln_kernels_time.py"""
import json
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from distributed_tensorflow_example_amd.ops import transformer as T  # noqa: E402


def timed(fn, iters=200):
    for _ in range(20):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    C = T._C()
    N, H, p, seed = 16384, 768, 0.1, -(1 << 63) + 12345   # bit 63 set: the 32-bit hash
    dev = "cuda"
    bf = dict(dtype=torch.bfloat16, device=dev)
    x, r, dy = (torch.randn(N, H, **bf) for _ in range(3))
    bias, gamma, beta = (torch.randn(H, device=dev) for _ in range(3))
    y, s, ds, dxb = (torch.empty(N, H, **bf) for _ in range(4))
    mean, rstd = torch.empty(N, device=dev), torch.empty(N, device=dev)
    dg, db, dbias = (torch.empty(H, device=dev) for _ in range(3))
    part = T._ln_part(N, H, dev)
    fwd = timed(lambda: C.bdrln_fwd(x, bias, r, gamma, beta, y, s, mean, rstd, 1e-12, p, seed))
    bwd = timed(lambda: C.ln_bwd(dy, s, mean, rstd, gamma, ds, dxb, part, dg, db, dbias, p, seed, False))
    mb = N * H * 2 / 1e6
    print(json.dumps({"tree": os.path.basename(os.getcwd()), "bdrln_fwd_us": round(fwd, 2),
                      "bdrln_fwd_TBps": round(4 * mb / fwd, 2), "ln_bwd_us": round(bwd, 2),
                      "ln_bwd_TBps": round(4 * mb / bwd, 2), "note": "ln_bwd time includes its colsum launch"}))


if __name__ == "__main__":
    main()
