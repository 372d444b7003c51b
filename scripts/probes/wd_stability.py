#!/usr/bin/env python3
"""Wide&Deep loss trajectory on the GPU, eager vs one-hipGraph step, on the
bench's data (scripts/bench_models.py: Zipf-1.1 ids, 16 cycled batches) and
hyper-parameters.  Prints one JSON line per mode: losses every 10 steps, the
largest |row| of each table and, at the first non-finite loss, where it shows
up first (tables, tower weights / grads, Adam slots, bag outputs).

    python scripts/probes/wd_stability.py STEPS F MODES [sparse_opt]
"""
from __future__ import annotations

import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_tensorflow_example_amd.models.wide_deep import WideDeep  # noqa: E402
from distributed_tensorflow_example_amd.parallel.world import World  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bench_models import synthetic_sparse_batches  # noqa: E402


def _stat(t):
    t = t.detach().reshape(-1)
    lo, hi = torch.aminmax(t)
    return {"nonfinite": int((~torch.isfinite(t)).sum()), "absmax": max(-float(lo), float(hi))}


def snapshot(m):
    out = {"wide": _stat(m.wide.local), "emb": _stat(m.emb.local),
           "step_t": int(m.opt.step_t.item()), "flat_grad": _stat(m.flat_grad)}
    for i, p in enumerate(m.layers):
        out[f"layer{i}"] = _stat(p.data)
    for i, (mm, vv) in enumerate(zip(m.opt.m, m.opt.v)):
        if mm is not None:
            out[f"adam_m{i}"] = _stat(mm)
            out[f"adam_v{i}"] = _stat(vv)
    return out


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 220
    F = int(float(sys.argv[2])) if len(sys.argv) > 2 else 10_000_000
    modes = sys.argv[3].split(",") if len(sys.argv) > 3 else ["eager", "graph"]
    sparse_opt = sys.argv[4] if len(sys.argv) > 4 else "sgd"
    B, nnz = 4096, 32
    dev = torch.device("cuda", 0)
    batches = synthetic_sparse_batches(16, B, F, nnz, 1234, dev)
    for mode in modes:
        torch.cuda.empty_cache()
        m = WideDeep(F, emb_dim=64, hidden=(512, 256), lr=0.05, dense_opt="adam", dense_lr=1e-3,
                     world=World(device=dev), ids_capacity=B * nnz if mode != "eager-exact" else None, rows=B,
                     sparse_opt=sparse_opt)
        init = snapshot(m)
        if mode == "graph":
            m.enable_graph()
        losses, first_bad, before = [], None, None
        for i in range(steps):
            prev = snapshot(m)
            loss = float(m.train_step(batches[i % len(batches)]))
            if i % 10 == 0 or i == steps - 1:
                losses.append(round(loss, 5))
            if first_bad is None and not math.isfinite(loss):
                first_bad = {"step": i, "after": snapshot(m), "before": prev}
                break
        print(json.dumps({"mode": mode, "F": F, "sparse_opt": sparse_opt, "init": init, "losses": losses,
                          "first_nonfinite": first_bad, "final": snapshot(m)}), flush=True)
        del m
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
