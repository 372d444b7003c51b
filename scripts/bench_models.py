"""Secondary benchmarks (BASELINE configs #3-#5 and the sparse LR workload).

    python scripts/bench_models.py --model wide_deep --steps 200 --warmup 20
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        scripts/bench_models.py --model wide_deep

Same timing contract as bench.py (barrier + synchronize around exactly K
timed steps, max over ranks, one JSON line from rank 0); synthetic inputs,
random-init weights.  The headline metric stays the MNIST MLP in bench.py.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def synthetic_sparse_batches(n_batches, batch, num_features, nnz, seed, device):
    """Power-law ids (Zipf 1.1) with `nnz` features per sample, CSR on device."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n_batches):
        ids = (rng.zipf(1.1, batch * nnz) - 1) % num_features
        vals = np.ones(batch * nnz, np.float32)
        offs = np.arange(0, batch * nnz + 1, nnz, dtype=np.int64)
        lab = (rng.random((batch, 1)) < 0.3).astype(np.float32)
        out.append(tuple(torch.from_numpy(a).to(device) for a in (lab, offs, ids.astype(np.int64), vals)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=["wide_deep", "sparse_lr"], default="wide_deep")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=4096, help="per-GPU batch")
    ap.add_argument("--features", type=int, default=100_000_000, help="table rows (sharded)")
    ap.add_argument("--emb-dim", type=int, default=64)
    ap.add_argument("--nnz", type=int, default=32, help="features per sample")
    ap.add_argument("--gpus", type=int, default=None)
    a = ap.parse_args()

    from distributed_tensorflow_example_amd.parallel import world as W

    w = W.init()
    dev = w.device
    if a.model == "wide_deep":
        from distributed_tensorflow_example_amd.models.wide_deep import WideDeep

        m = WideDeep(a.features, emb_dim=a.emb_dim, hidden=(512, 256), lr=0.05, dense_opt="adam",
                     dense_lr=1e-3, world=w)
        cfg = {"model": f"wide_deep F={a.features} D={a.emb_dim} tower=512-256-1", "global_batch": a.batch * w.world_size,
               "per_gpu_batch": a.batch, "seq_len": None, "parallelism": f"dp{w.world_size}+emb-shard{w.world_size}",
               "nnz_per_sample": a.nnz}
    else:
        from distributed_tensorflow_example_amd.models.sparse_lr import SparseLRTrainer

        m = SparseLRTrainer(a.features, 0.1, w)
        cfg = {"model": f"sparse_lr F={a.features}", "global_batch": a.batch * w.world_size, "per_gpu_batch": a.batch,
               "seq_len": None, "parallelism": f"emb-shard{w.world_size}", "nnz_per_sample": a.nnz}
    batches = synthetic_sparse_batches(16, a.batch, a.features, a.nnz, 1234 + w.rank, dev)
    for i in range(a.warmup):
        m.train_step(batches[i % len(batches)])
    w.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.time()
    for i in range(a.steps):
        loss = m.train_step(batches[i % len(batches)])
    if dev.type == "cuda":
        torch.cuda.synchronize()
    w.barrier()
    dt = w.host_all_reduce(time.time() - t0, "max")
    sps = a.batch * w.world_size * a.steps / dt
    if w.rank == 0:
        print(json.dumps({"metric": f"{a.model} samples/sec (whole node)", "value": round(sps, 1),
                          "unit": "samples/s", "n_gpus": w.world_size, "steps": a.steps, "warmup": a.warmup,
                          "ms_per_step": round(dt / a.steps * 1e3, 4), "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic zipf ids",
                          "config": cfg, "final_loss": float(loss)}), flush=True)
    w.shutdown()


if __name__ == "__main__":
    main()
