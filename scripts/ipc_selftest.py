"""Functional self-test of the one-shot IPC all-reduce (models.mlp, ipc path).

Launch: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
            scripts/ipc_selftest.py [--same-gpu]
Runs K fused MLP steps with the IPC reduce-apply on every rank (gloo control
plane; with --same-gpu all ranks share cuda:0, which exercises the IPC
mapping, flags and double-buffered slots on a 1-GPU box) and checks:
  * no in-kernel wait timed out;
  * replicas are bit-identical across ranks;
  * the result matches a single-process fp32 reference of the same global
    batch (mean of the per-rank gradients) within bf16 tolerance.
Prints one JSON line from rank 0; exit code 0 on success.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--same-gpu", action="store_true")
    ap.add_argument("--ipc-timeout", type=float, default=30.0,
                    help="in-kernel wait bound per exchange (s); ranks sharing one GPU are time-sliced")
    ap.add_argument("--graph", action="store_true", help="also replay the steps from a captured hipGraph")
    a = ap.parse_args()
    rank, ws = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    from distributed_tensorflow_example_amd.models import mlp
    from distributed_tensorflow_example_amd.parallel.world import World

    dev = torch.device("cuda", 0 if a.same_gpu else rank % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=ws,
                            timeout=datetime.timedelta(seconds=120))
    w = World(rank=rank, world_size=ws, local_rank=rank, device=dev, backend="gloo", pg_initialized=True)
    tr = mlp.FusedMLPTrainer(batch_size=100, lr=0.05, world=w, device=dev, allreduce=os.environ.get("DTF_IPC_MODE", "ipc-fused"), ipc_timeout_s=a.ipc_timeout)
    g = torch.Generator().manual_seed(7)
    xs = torch.randint(0, 256, (a.steps, ws, 100, 784), generator=g, dtype=torch.uint8)
    ys = torch.randint(0, 10, (a.steps, ws, 100), generator=g)
    ref = mlp.init_params(1).clone()
    # start the first exchange together: a rank still paging in torch/HIP on a
    # cold box must not eat the peers' in-kernel wait budget
    torch.cuda.synchronize()
    dist.barrier()
    for s in range(a.steps):
        tr.step_tensors(xs[s, rank].to(dev), ys[s, rank].to(dev))
        # reference: mean over ranks of per-rank mean gradients == one 200-row batch
        gsum = torch.zeros_like(ref)
        for r in range(ws):
            _, _, gr = mlp.reference_loss_and_grad(ref, xs[s, r].float() / 255.0, ys[s, r])
            gsum += gr
        ref -= 0.05 * gsum / ws
    torch.cuda.synchronize()
    err = tr.ipc_error()
    p = tr.params.detach().cpu().double()
    sums = [None] * ws
    dist.all_gather_object(sums, (float(p.sum()), float(p.abs().sum()), err))
    identical = len({(a_, b_) for a_, b_, _ in sums}) == 1
    rel = float((p - ref.double()).norm() / ref.double().norm())
    ok = identical and all(e == 0 for _, _, e in sums) and rel < 2e-3
    if rank == 0:
        print(json.dumps({"ipc_selftest": "pass" if ok else "FAIL", "world": ws, "same_gpu": a.same_gpu,
                          "steps": a.steps, "identical_replicas": identical, "rel_err_vs_fp32_ref": rel,
                          "ipc_errors": [e for _, _, e in sums]}), flush=True)
    dist.barrier()
    tr.ipc.close()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
