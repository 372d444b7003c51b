"""Cost of the prob-dropout hash inside the fused attention kernels: BERT-base
layer shape (B=128, S=128, 12 heads, d=64), forward + backward with p = 0.1 vs
p = 0 (CUDA events, median of 5 x 20 calls).  Prints one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_tensorflow_example_amd.ops import transformer as T  # noqa: E402


def main():
    B, S, NH, d = 128, 128, 12, 64
    dev = torch.device("cuda")
    qkv = (torch.randn(B, S, 3 * NH * d, device=dev) * 0.5).to(torch.bfloat16).requires_grad_(True)
    bias = torch.randn(3 * NH * d, device=dev) * 0.1
    mask = torch.zeros(B, S, device=dev)
    g = torch.randn(B, S, NH * d, device=dev).to(torch.bfloat16)
    out = {}
    for p in (0.1, 0.0):
        def fwd():
            return T.fused_attention(qkv, bias, mask, NH, 0.125, p)
        for _ in range(3):
            fwd().backward(g)
        ts_f, ts_b = [], []
        for _ in range(5):
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            ys = []
            e0.record()
            for _ in range(20):
                ys.append(fwd())
            e1.record()
            for y in ys:
                y.backward(g)
            e2.record()
            torch.cuda.synchronize()
            ts_f.append(e0.elapsed_time(e1) / 20 * 1e3)
            ts_b.append(e1.elapsed_time(e2) / 20 * 1e3)
        ts_f.sort()
        ts_b.sort()
        out[f"p{p}"] = {"fwd_us": round(ts_f[2], 2), "bwd_us": round(ts_b[2], 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
