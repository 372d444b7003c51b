#!/usr/bin/env python3
"""Per-launch timing of the large-batch MLP step (mlp_gemm.hip): the forward
(mlpg_l1 + mlpg_head), mlpg_wgrad, mlpg_apply and the whole step.  One JSON line
per (B, item): us per launch over back-to-back launches (events)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_tensorflow_example_amd.data.mnist import synthetic_mnist  # noqa: E402
from distributed_tensorflow_example_amd.models import mlp  # noqa: E402


def timeit(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / n


def main():
    dev = torch.device("cuda", 0)
    for B in (1024, 4096):
        imgs, labels = synthetic_mnist(B, seed=2)
        x = torch.from_numpy(imgs).to(dev).contiguous().view(-1)
        y = torch.from_numpy(labels).to(dev)
        tr = mlp.GemmMLPTrainer(batch_size=B, device=dev)
        C = tr.C
        out = {"B": B, "nchunk": tr.nchunk}
        out["fwd_us"] = round(timeit(lambda: C.mlpg_fwd(x, 0, y, 0, B, tr.W1S, tr.params, tr.a2, tr.P1, tr.dz2S,
                                                       tr.act, False, 1.0 / B)), 2)
        out["wgrad_us"] = round(timeit(lambda: C.mlpg_wgrad(x, 0, B, tr.dz2S, tr.P2, tr.nchunk)), 2)
        out["apply_us"] = round(timeit(lambda: tr._apply(0)), 2)
        out["step_us"] = round(timeit(lambda: tr.enqueue_step(x, 0, 0, y, 0)), 2)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
