"""Hogwild parameter store over IPC (parallel/async_ps.py, csrc/kernels/hogwild.hip)
with N ranks: every rank applies `steps` integer-valued updates of its own to the
variables hosted in rank 0's device memory, without waiting for the others.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        scripts/async_ps_selftest.py [--same-gpu] [--no-locking]

Prints one JSON line: with locking every update lands (exact final values);
global steps 1..N*steps are handed out exactly once either way.
"""
import argparse
import datetime
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--same-gpu", action="store_true")
    ap.add_argument("--no-locking", action="store_true")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--table", action="store_true",
                    help="a row-sharded table (HogwildTable): rows read from / scatter-updated into the owners' "
                         "IPC-mapped shards")
    a = ap.parse_args()
    from distributed_tensorflow_example_amd.parallel import async_ps
    from distributed_tensorflow_example_amd.parallel.world import World

    rank, ws = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0 if a.same_gpu else rank % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=ws,
                            timeout=datetime.timedelta(seconds=120))
    w = World(rank=rank, world_size=ws, local_rank=rank, device=dev, backend="gloo", pg_initialized=True)
    if a.table:
        return table_test(a, w, dev, rank, ws)
    n = 79510                                  # the MLP's parameter count
    p1 = torch.full((n - 10,), 1000.0, device=dev) if rank == 0 else torch.zeros(n - 10, device=dev)
    p2 = torch.full((10,), 1000.0, device=dev) if rank == 0 else torch.zeros(10, device=dev)
    st = async_ps.HogwildStore([p1, p2], w, use_locking=not a.no_locking)
    st.pull()
    init_ok = bool((p1 == 1000.0).all().item() and (p2 == 1000.0).all().item())
    w.barrier()
    gsteps = []
    for _ in range(a.steps):
        g = [torch.full_like(p1, float(rank + 1)), torch.full_like(p2, float(rank + 1))]
        gsteps.append(st.sgd_step(g, 1.0))
    torch.cuda.synchronize()
    w.barrier()
    st.pull()
    torch.cuda.synchronize()
    final = float(p1[0].item()), float(p1[-1].item()), float(p2[5].item())
    allg = w.all_gather_object(gsteps)
    total = st.global_step()
    expect = 1000.0 - a.steps * ws * (ws + 1) / 2
    steps_ok = sorted(sum(allg, [])) == list(range(1, ws * a.steps + 1)) and total == ws * a.steps
    if a.no_locking:
        vals_ok = all(expect <= v <= 1000.0 - a.steps for v in final)
    else:
        vals_ok = all(v == expect for v in final)
    st.close()
    if rank == 0:
        print(json.dumps({"async_ps_selftest": "pass" if (init_ok and steps_ok and vals_ok) else "fail",
                          "kind": st.kind, "final": final, "expect": expect, "global_step": total,
                          "init_ok": init_ok, "steps_ok": steps_ok}), flush=True)
    dist.destroy_process_group()


def table_test(a, w, dev, rank, ws):
    """Every rank scatter-SGDs its own gradient (rank + 1) into the same 64 rows
    of a 1003 x 4 table spread over all shards (every owner, odd local rows),
    `steps` times, without waiting; with locking every update lands."""
    from distributed_tensorflow_example_amd.parallel import async_ps
    from distributed_tensorflow_example_amd.parallel.sharded_embedding import ShardedEmbedding

    F, D = 1003, 4
    t = ShardedEmbedding(F, D, w, device=dev, zero_init=True, name="tab")
    with torch.no_grad():
        t.local.fill_(1000.0)
    hog = async_ps.HogwildTable(t, w, use_locking=not a.no_locking)
    t.hogwild = hog
    ids = torch.arange(5, 5 + 64 * 7, 7, device=dev)
    rows, ctx = t.lookup(ids)
    init_ok = bool((rows == 1000.0).all().item()) and ctx.hogwild
    w.barrier()
    for _ in range(a.steps):
        rows, ctx = t.lookup(ids)
        t.apply_sgd(ctx, torch.full((ctx.uniq.numel(), D), float(rank + 1), device=dev), 1.0)
    torch.cuda.synchronize()
    w.barrier()
    rows, _ = t.lookup(ids)
    others, _ = t.lookup(torch.arange(6, 6 + 64 * 7, 7, device=dev))     # never updated
    torch.cuda.synchronize()
    expect = 1000.0 - a.steps * ws * (ws + 1) / 2
    if a.no_locking:
        vals_ok = bool(((rows >= expect) & (rows <= 1000.0 - a.steps)).all().item())
    else:
        vals_ok = bool((rows == expect).all().item())
    untouched = bool((others == 1000.0).all().item())
    full = t.full_table()
    shard_ok = bool((full[ids] == rows).all().item())
    kind = hog.kind
    hog.close()
    if rank == 0:
        ok = init_ok and vals_ok and untouched and shard_ok
        print(json.dumps({"async_ps_selftest": "pass" if ok else "fail", "kind": kind, "table": True, "final": float(rows[0, 0].item()), "expect": expect,
                          "init_ok": init_ok, "vals_ok": vals_ok, "untouched": untouched, "shard_ok": shard_ok}),
              flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
