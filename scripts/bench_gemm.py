#!/usr/bin/env python3
"""gemm_big.hip vs torch (hipBLASLt) on BERT-base's linear-layer products.

T = B*S tokens (default 128 x 128); every linear of a BERT layer in its three
roles (forward, input gradient, weight gradient) on random normal bf16 data,
variants interleaved in one process (rounds x reps), median ms and TFLOP/s.
"ours" is the automatic schedule (8-phase when K % 128 == 0), "ours_v4" the
one-barrier loop it replaced.  The weight gradient is also timed the way models/bert.py ran it before
(token-slab bmm + slab_sum).  One JSON line per (layer, role).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_example_amd import _native  # noqa: E402
from distributed_tensorflow_example_amd.models import bert  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=128 * 128)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    C = _native.load()
    T = a.tokens
    dev = torch.device("cuda", 0)
    layers = {"qkv": (2304, 768), "attn_out": (768, 768), "ffn1": (3072, 768), "ffn2": (768, 3072)}
    for name, (O, I) in layers.items():
        x = torch.randn(T, I, device=dev).bfloat16()
        w = (torch.randn(O, I, device=dev) * 0.05).bfloat16()
        gy = torch.randn(T, O, device=dev).bfloat16()
        y = torch.empty(T, O, device=dev, dtype=torch.bfloat16)
        gx = torch.empty(T, I, device=dev, dtype=torch.bfloat16)
        dw = torch.zeros(O, I, device=dev)
        roles = {
            "fwd": {"ours": lambda: C.gemm_big(x, False, w, True, y),
                    "ours_v4": lambda: C.gemm_big(x, False, w, True, y, variant=4),
                    "torch": lambda: torch.mm(x, w.t(), out=y)},
            "dx": {"ours": lambda: C.gemm_big(gy, False, w, False, gx),
                   "ours_v4": lambda: C.gemm_big(gy, False, w, False, gx, variant=4),
                   "torch": lambda: torch.mm(gy, w, out=gx)},
            # input gradient accumulated onto a residual branch's (beta = 1), as models/bert.py runs it
            "dx_res": {"ours": lambda: C.gemm_big(gy, False, w, False, gx, beta=1.0),
                       "ours_v4": lambda: C.gemm_big(gy, False, w, False, gx, beta=1.0, variant=4),
                       "torch": lambda: gx.addmm_(gy, w)},
            "dw": {"ours": lambda: C.gemm_big(gy, True, x, False, dw, beta=1.0, split_k=0),
                   "ours_v4": lambda: C.gemm_big(gy, True, x, False, dw, beta=1.0, split_k=0, variant=4),
                   "torch": lambda: torch.addmm(dw, gy.t(), x, out_dtype=torch.float32, out=dw),
                   "torch_slabs": lambda: bert._wgrad(gy, x, into=dw)},
        }
        for role, fns in roles.items():
            M, N, K = {"fwd": (T, O, I), "dx": (T, I, O), "dx_res": (T, I, O), "dw": (O, I, T)}[role]
            flop = 2.0 * M * N * K
            times = {k: [] for k in fns}
            for f in fns.values():
                f()
            torch.cuda.synchronize()
            for _ in range(a.rounds):
                for k, f in fns.items():
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(a.reps):
                        f()
                    e.record()
                    e.synchronize()
                    times[k].append(s.elapsed_time(e) / a.reps)
            out = {"layer": name, "role": role, "M": M, "N": N, "K": K}
            for k, v in times.items():
                med = statistics.median(v)
                out[k + "_ms"] = round(med, 4)
                out[k + "_tflops"] = round(flop / med / 1e9, 1)
            out["speedup_vs_best_torch"] = round(min(out[k + "_ms"] for k in fns if not k.startswith("ours")) / out["ours_ms"], 3)
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
