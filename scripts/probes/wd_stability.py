#!/usr/bin/env python3
"""Wide&Deep loss trajectory on the GPU, eager vs one-hipGraph step, on the
bench's data (scripts/bench_models.py: Zipf-1.1 ids, 16 cycled batches) and
hyper-parameters, with a smaller table.  Prints one JSON line per mode:
losses every 20 steps and the largest |row| of each table."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_tensorflow_example_amd.models.wide_deep import WideDeep  # noqa: E402
from distributed_tensorflow_example_amd.parallel.world import World  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bench_models import synthetic_sparse_batches  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 220
    F = int(float(sys.argv[2])) if len(sys.argv) > 2 else 10_000_000
    modes = sys.argv[3].split(",") if len(sys.argv) > 3 else ["eager", "graph"]
    B, nnz = 4096, 32
    dev = torch.device("cuda", 0)
    batches = synthetic_sparse_batches(16, B, F, nnz, 1234, dev)
    for mode in modes:
        m = WideDeep(F, emb_dim=64, hidden=(512, 256), lr=0.05, dense_opt="adam", dense_lr=1e-3,
                     world=World(device=dev), ids_capacity=B * nnz, rows=B)
        init = {"emb_finite": bool(torch.isfinite(m.emb.local).all()), "emb_max": float(m.emb.local.abs().max()),
                "emb_std_tail": float(m.emb.local[-1000:].std()), "wide_max": float(m.wide.local.abs().max())}
        if mode == "graph":
            m.enable_graph()
        losses = []
        for i in range(steps):
            loss = m.train_step(batches[i % len(batches)])
            if i % 10 == 0 or i == steps - 1:
                losses.append(round(float(loss), 5))
        print(json.dumps({"mode": mode, "F": F, "init": init, "losses": losses,
                          "wide_max": float(m.wide.local.abs().max()), "emb_max": float(m.emb.local.abs().max())}),
              flush=True)


if __name__ == "__main__":
    main()
