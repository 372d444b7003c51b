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
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def _exchange_stats(m):
    """Static all-to-all per-peer capacity and wire ratio vs an exact exchange (W > 1)."""
    tab = getattr(m, "wide", None) or getattr(m, "W", None)
    r = getattr(tab, "router", None)
    if r is None or r.W == 1:
        return None
    wr = r.wire_ratio()
    return {"peer_capacity": r.peer_cap, "checks": r.checks, "resizes": r.resizes, "voided_steps": r.voided,
            "wire_ids_over_exact": None if wr is None else round(wr, 3)}


def refuse_diverged(w, loss, metric):
    """A run whose final loss is not finite is not a measurement: no value line,
    non-zero exit (collective: every rank exits alike)."""
    bad = 0.0 if math.isfinite(float(loss)) else 1.0
    if w.world_size > 1:
        bad = w.host_all_reduce(bad, "max")
    if bad:
        if w.rank == 0:
            print(json.dumps({"metric": metric, "error": "non-finite final loss; result discarded",
                              "final_loss": float(loss)}), file=sys.stderr, flush=True)
        w.shutdown()
        raise SystemExit(3)


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
    ap.add_argument("--model", choices=["wide_deep", "sparse_lr", "lr2", "bert_base", "resnet50"], default="wide_deep",
                    help="lr2 = sparse_lr at the reference's product configuration (run_lr2.sh:55-61: "
                         "F=1e9 features, batch 500, learning rate 1.0)")
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--bucket-mb", default="auto",
                    help="DDP bucket size in MB of fp32 gradient, auto (xGMI cost model) or measure (timed all-reduces; parallel/ddp.py)")
    ap.add_argument("--bucket-sweep", default="",
                    help="dense models: comma-separated bucket sizes in MB (e.g. 1,4,16,64) re-timed after the main "
                         "run; ms/step per size lands in the JSON line (xGMI bucket sizing, SURVEY s5.8)")
    ap.add_argument("--comm-bf16", action="store_true", help="dense models: bf16 gradient all-reduce (BASELINE #2)")
    ap.add_argument("--no-shadow", action="store_true", help="cast fp32 weights per GEMM/conv (autocast) instead of bf16 shadows")
    ap.add_argument("--conv-find", type=int, default=1,
                    help="ResNet: 1 = let MIOpen benchmark conv solvers (torch.backends.cudnn.benchmark)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=0, help="per-GPU batch (0 = model default)")
    ap.add_argument("--features", type=int, default=100_000_000, help="table rows (sharded)")
    ap.add_argument("--emb-dim", type=int, default=64)
    ap.add_argument("--nnz", type=int, default=32, help="features per sample")
    ap.add_argument("--gpus", type=int, default=None)
    ap.add_argument("--lr", type=float, default=None, help="sparse models: SGD learning rate")
    ap.add_argument("--sparse-opt", default="sgd", choices=["sgd", "adagrad", "momentum", "rmsprop", "adam"],
                    help="wide_deep: the tables' owner-side update rule")
    ap.add_argument("--graph", action="store_true", help="sparse_lr / lr2 / wide_deep: replay each step as one captured hipGraph")
    ap.add_argument("--trace-marker", action="store_true",
                    help="launch a spin kernel right before the timed loop, so a kernel trace can be cut to the "
                         "steady state (scripts/rocpd_summary.py --after spin)")
    a = ap.parse_args()
    if a.model == "lr2":
        a.features = a.features if a.features != 100_000_000 else 1_000_000_000
        a.batch = a.batch or 500
        a.lr = 1.0 if a.lr is None else a.lr
        a.nnz = a.nnz if a.nnz != 32 else 40

    from distributed_tensorflow_example_amd.parallel import world as W

    w = W.init()
    dev = w.device
    if a.model in ("bert_base", "resnet50"):
        return dense_bench(a, w)
    a.batch = a.batch or 4096
    if dev.type == "cuda":
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats()
    t_init = time.time()
    if a.model == "wide_deep":
        from distributed_tensorflow_example_amd.models.wide_deep import WideDeep

        m = WideDeep(a.features, emb_dim=a.emb_dim, hidden=(512, 256), lr=0.05, dense_opt="adam",
                     dense_lr=1e-3, world=w, ids_capacity=a.batch * a.nnz if (a.graph or w.world_size > 1) else None,
                     rows=a.batch, sparse_opt=a.sparse_opt)
        if a.graph:
            m.enable_graph()
        cfg = {"model": f"wide_deep F={a.features} D={a.emb_dim} tower=512-256-1", "global_batch": a.batch * w.world_size,
               "per_gpu_batch": a.batch, "seq_len": None, "parallelism": f"dp{w.world_size}+emb-shard{w.world_size}",
               "nnz_per_sample": a.nnz, "graph": bool(a.graph), "sparse_opt": a.sparse_opt}
    else:
        from distributed_tensorflow_example_amd.models.sparse_lr import SparseLRTrainer

        m = SparseLRTrainer(a.features, 0.1 if a.lr is None else a.lr, w, ids_capacity=a.batch * a.nnz, rows=a.batch)
        if a.graph:
            m.enable_graph()
        cfg = {"model": f"{'lr2 ' if a.model == 'lr2' else ''}sparse_lr F={a.features}",
               "global_batch": a.batch * w.world_size, "per_gpu_batch": a.batch, "lr": 0.1 if a.lr is None else a.lr,
               "seq_len": None, "parallelism": f"emb-shard{w.world_size}", "nnz_per_sample": a.nnz,
               "graph": bool(a.graph)}
    if dev.type == "cuda":
        torch.cuda.synchronize()
    init_s = time.time() - t_init
    init_mem = torch.cuda.max_memory_allocated() / 2 ** 30 if dev.type == "cuda" else None
    batches = synthetic_sparse_batches(16, a.batch, a.features, a.nnz, 1234 + w.rank, dev)
    for i in range(a.warmup):
        m.train_step(batches[i % len(batches)])
    w.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
        if a.trace_marker:
            torch.cuda._sleep(1000)
            torch.cuda.synchronize()
    t0 = time.time()
    for i in range(a.steps):
        loss = m.train_step(batches[i % len(batches)])
    if dev.type == "cuda":
        torch.cuda.synchronize()
    w.barrier()
    dt = w.host_all_reduce(time.time() - t0, "max")
    sps = a.batch * w.world_size * a.steps / dt
    refuse_diverged(w, loss, f"{a.model} samples/sec (whole node)")
    if w.rank == 0:
        print(json.dumps({"metric": f"{a.model} samples/sec (whole node)", "value": round(sps, 1),
                          "unit": "samples/s", "n_gpus": w.world_size, "steps": a.steps, "warmup": a.warmup,
                          "ms_per_step": round(dt / a.steps * 1e3, 4), "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic zipf ids",
                          "config": cfg, "final_loss": float(loss), "init_s": round(init_s, 3),
                          "init_peak_mem_gib": None if init_mem is None else round(init_mem, 3),
                          "sparse_exchange": _exchange_stats(m),
                          "data_plane": {"ipc_calls": int(w.ipc.calls()) if w.ipc is not None else 0,
                                         "rccl_comm": w.comm is not None},
                          "peak_mem_gib": round(torch.cuda.max_memory_allocated() / 2 ** 30, 3)
                          if dev.type == "cuda" else None}), flush=True)
    w.shutdown()


def dense_bench(a, w):
    """BERT-base MLM / ResNet-50 with bucketed DDP (comm overlapped with backward)."""
    from distributed_tensorflow_example_amd import optim
    from distributed_tensorflow_example_amd.parallel.ddp import DistributedDataParallel

    dev = w.device
    if a.model == "bert_base":
        from distributed_tensorflow_example_amd.models.bert import BertConfig, BertForMLM, synthetic_mlm_batch

        a.batch = a.batch or 32
        model = BertForMLM(BertConfig.base(), seed=0).to(dev)
        batches = [synthetic_mlm_batch(a.batch, a.seq, 30522, dev, seed=w.rank * 100 + i) for i in range(4)]
        opt = optim.FusedAdamW(list(model.parameters()), 1e-4, weight_decay=0.01)
        unit, per = "sequences/s", a.batch
        cfg = {"model": "bert-base-uncased MLM (110M)", "global_batch": a.batch * w.world_size,
               "per_gpu_batch": a.batch, "seq_len": a.seq, "parallelism": f"dp{w.world_size}",
               "optimizer": "adamw", "grad_allreduce": f"bucketed {a.bucket_mb}MB, overlapped"}
        run = lambda m, b: m(*b)
    else:
        from distributed_tensorflow_example_amd.models.resnet import resnet50, synthetic_imagenet_batch

        a.batch = a.batch or 128
        torch.backends.cudnn.benchmark = bool(a.conv_find)
        model = resnet50().to(dev).to(memory_format=torch.channels_last)
        batches = [synthetic_imagenet_batch(a.batch, dev, seed=w.rank * 100 + i) for i in range(2)]
        opt = optim.FusedMomentum(list(model.parameters()), 0.1, 0.9, weight_decay=1e-4)
        unit, per = "images/s", a.batch
        cfg = {"model": "resnet50 (25.6M)", "global_batch": a.batch * w.world_size, "per_gpu_batch": a.batch,
               "seq_len": None, "parallelism": f"dp{w.world_size}", "optimizer": "sgd-momentum",
               "grad_allreduce": f"bucketed {a.bucket_mb}MB, overlapped", "input": "224x224 synthetic, channels_last",
               "conv_solver_search": bool(a.conv_find)}
        run = lambda m, b: m.loss(*b)
    comm_dtype = torch.bfloat16 if a.comm_bf16 else None
    ddp = DistributedDataParallel(model, w, bucket_mb=a.bucket_mb if a.bucket_mb in ("auto", "measure") else float(a.bucket_mb),
                                  comm_dtype=comm_dtype)
    cfg["grad_allreduce"] = f"bucketed {ddp.bucket_mb:.1f}MB x {len(ddp.buckets)} ({a.bucket_mb}), overlapped"
    if ddp.comm_cost:
        cfg["allreduce_alpha_us"] = round(ddp.comm_cost[0] * 1e6, 2)
        cfg["allreduce_GBps"] = round(ddp.comm_cost[1] / 1e9, 2)
    if not a.no_shadow:
        model.attach_shadows(opt)          # after the DDP broadcast: shadows match rank 0's weights

    def step(b):
        ddp.zero_grad()
        ddp.reset_step()
        loss = run(model, b)
        loss.backward()
        ddp.finish_gradient_synchronization()
        opt.step()
        return loss

    for i in range(a.warmup):
        step(batches[i % len(batches)])
    w.barrier()
    torch.cuda.synchronize()
    t0 = time.time()
    for i in range(a.steps):
        loss = step(batches[i % len(batches)])
    torch.cuda.synchronize()
    w.barrier()
    dt = w.host_all_reduce(time.time() - t0, "max")
    v = per * w.world_size * a.steps / dt
    refuse_diverged(w, loss, f"{a.model} {unit} (whole node)")
    sweep = {}
    for mb in [float(x) for x in a.bucket_sweep.split(",") if x.strip()]:
        ddp.close()
        ddp = DistributedDataParallel(model, w, bucket_mb=mb, comm_dtype=comm_dtype, broadcast_params=False)
        for i in range(3):
            step(batches[i % len(batches)])
        w.barrier()
        torch.cuda.synchronize()
        t1 = time.time()
        n = max(1, a.steps // 2)
        for i in range(n):
            step(batches[i % len(batches)])
        torch.cuda.synchronize()
        w.barrier()
        sweep[str(mb)] = {"ms_per_step": round(w.host_all_reduce(time.time() - t1, "max") / n * 1e3, 3),
                          "buckets": len(ddp.buckets)}
    if w.rank == 0:
        out = {"metric": f"{a.model} {unit} (whole node)", "value": round(v, 2), "unit": unit,
               "n_gpus": w.world_size, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 3),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
               "data": "synthetic", "config": cfg, "final_loss": float(loss)}
        if a.model == "resnet50":
            from distributed_tensorflow_example_amd.ops import conv as conv_ops
            # which engine each conv product runs on (per-shape timing), with the timed ms
            out["conv_engines"] = {f"{k[0]}:{'x'.join(map(str, k[1]))}->{k[2]}" + (f"/s{k[3]}" if len(k) > 3 else ""):
                                   [e, t] for k, (e, t) in conv_ops.choices().items()}
        if a.model == "bert_base":
            out["tokens_per_s"] = round(v * a.seq, 1)
            from distributed_tensorflow_example_amd.ops import big_gemm
            ch = big_gemm.choices()
            out["config"]["linear_gemm_policy"] = big_gemm.policy()
            if ch:   # which linear products ran on gemm_big.hip (auto: timed per shape)
                out["config"]["linear_gemm_native"] = {f"{k[0]}:{k[1]}x{k[2]}x{k[3]}": v[0] for k, v in ch.items()}
        if sweep:
            out["bucket_sweep"] = sweep
        out["config"]["grad_comm_dtype"] = "bf16" if a.comm_bf16 else "fp32"
        print(json.dumps(out), flush=True)
    w.shutdown()


if __name__ == "__main__":
    main()
