#!/usr/bin/env python3
"""Fixed vs per-K cost of gemm_big's schedules: forward layout (x W^T, bf16
out) at M = 16384 tokens, N in {768, 3072}, K swept 256 .. 6144.  A linear
fit of time against K gives the per-K-tile loop cost (slope) and the
per-output-tile overhead (intercept: prologue, epilogue, dispatch); torch
(hipBLASLt) is timed alongside.  One JSON line per (N, K)."""
from __future__ import annotations

import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_tensorflow_example_amd import _native  # noqa: E402


def timed(f, reps=10, rounds=5):
    f()
    torch.cuda.synchronize()
    out = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            f()
        e.record()
        e.synchronize()
        out.append(s.elapsed_time(e) / reps)
    return statistics.median(out)


def main():
    C = _native.load()
    M = 16384
    for N in (768, 3072):
        for K in (256, 512, 768, 1536, 3072, 6144):
            x = torch.randn(M, K, device="cuda").bfloat16()
            w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
            y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            row = {"M": M, "N": N, "K": K}
            for name, f in (("v8", lambda: C.gemm_big(x, False, w, True, y, variant=8)),
                            ("v8_w192", lambda: C.gemm_big_cfg(14, x, w, y)),
                            ("v8_noepi", lambda: C.gemm_big_cfg(11, x, w, y)),
                            ("v8_quarter", lambda: C.gemm_big_cfg(12, x, w, y)),
                            ("v8_samedst", lambda: C.gemm_big_cfg(13, x, w, y)),
                            ("v4", lambda: C.gemm_big(x, False, w, True, y, variant=4)),
                            ("torch", lambda: torch.mm(x, w.t(), out=y))):
                ms = timed(f)
                row[name + "_us"] = round(ms * 1e3, 2)
                row[name + "_tflops"] = round(2.0 * M * N * K / ms / 1e9, 1)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
