"""Probe: BERT weight-gradient GEMM variants (hipBLASLt) at T = B*S tokens.

gw[out, in] = gy[T, out]^T @ x[T, in]; master grads are fp32.  hipBLASLt picks
non-split-K tiles for this long-K / small-MN shape; the split variants cut T
into S slabs, run one batched GEMM (S x the tiles) and reduce the slabs.
"""
import time

import torch


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.time()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.time() - t) / it * 1e6


T = 16384
for out, inp in [(2304, 768), (768, 768), (3072, 768), (768, 3072)]:
    gy = torch.randn(T, out, device="cuda").bfloat16()
    x = torch.randn(T, inp, device="cuda").bfloat16()
    g = torch.zeros(out, inp, device="cuda")
    fl = 2 * T * out * inp
    res = {"mm_f32out": timeit(lambda: torch.mm(gy.t(), x, out_dtype=torch.float32))}
    ref = torch.mm(gy.t(), x, out_dtype=torch.float32)
    for S in (2, 4, 8, 16):
        gys = gy.view(S, T // S, out).transpose(1, 2)
        xs = x.view(S, T // S, inp)

        def f32():
            g.add_(torch.bmm(gys, xs, out_dtype=torch.float32).sum(0))

        def b16():
            g.add_(torch.bmm(gys, xs).sum(0, dtype=torch.float32))
        try:
            res[f"bmm{S}_f32+sum"] = timeit(f32)
        except Exception as e:
            res[f"bmm{S}_f32+sum"] = float("nan")
            print("f32 bmm failed", e)
        res[f"bmm{S}_bf16+sum"] = timeit(b16)
        if S == 4:
            g.zero_()
            f32()
            print("  split4 rel err", float((g - ref).norm() / ref.norm()))
    print(f"out={out} in={inp}: " + "  ".join(f"{k} {v:.1f}us ({fl / v / 1e6:.0f} TF/s)" for k, v in res.items()), flush=True)
