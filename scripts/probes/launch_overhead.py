"""Where the fixed cost of a short persistent run goes: host call, launch ->
kernel start, kernel body, completion -> synchronize return (bench.py times
run(20) between two synchronizes).

    python scripts/probes/launch_overhead.py [precision]
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from distributed_tensorflow_example_amd.data.mnist import PinnedEpoch, synthetic_mnist  # noqa: E402
from distributed_tensorflow_example_amd.models.mlp import FusedMLPTrainer, PersistentMLPRunner  # noqa: E402


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "fp32"
    dev = torch.device("cuda", 0)
    imgs, labels = synthetic_mnist(55000, seed=0)
    tr = FusedMLPTrainer(batch_size=100, lr=0.0005, device=dev)
    ep = PinnedEpoch(imgs, labels, 100)
    run = PersistentMLPRunner(tr, ep, steps_per_launch=550, precision=prec)
    run.prepare(550)
    run.run(550)
    torch.cuda.synchronize()
    x = torch.zeros(1, device=dev)
    out = {}
    for n in (20, 1):
        host, wall, ev_us, dev_us = [], [], [], []
        for rep in range(30):
            run.prepare(n)
            torch.cuda.synchronize()
            s0 = tr.global_step
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record()
            run.run(n)
            t1 = time.perf_counter()
            e1.record()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            host.append((t1 - t0) * 1e6)
            wall.append((t2 - t0) * 1e6)
            ev_us.append(e0.elapsed_time(e1) * 1e3)
            dev_us.append(float(run.step_times_ms(s0, s0 + n).sum()) * 1e3)
        med = lambda v: round(float(np.median(v)), 2)
        out[f"run_{n}"] = {"host_call_us": med(host), "wall_sync_to_sync_us": med(wall), "event_us": med(ev_us),
                           "device_steps_us": med(dev_us)}
    tiny = []
    for rep in range(30):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        x.add_(1.0)
        torch.cuda.synchronize()
        tiny.append((time.perf_counter() - t0) * 1e6)
    out["tiny_kernel_sync_to_sync_us"] = round(float(np.median(tiny)), 2)
    t = []
    for rep in range(30):
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        t.append((time.perf_counter() - t0) * 1e6)
    out["idle_synchronize_us"] = round(float(np.median(t)), 2)
    print(json.dumps(out))


if __name__ == "__main__" and not os.environ.get("BENCH_LIKE"):
    main()


def bench_like():
    """bench.py's exact sequence around its timed run(20), repeated, with and
    without an idle gap (host sleep) before t0."""
    dev = torch.device("cuda", 0)
    imgs, labels = synthetic_mnist(55000, seed=0)
    tr = FusedMLPTrainer(batch_size=100, lr=0.0005, device=dev)
    ep = PinnedEpoch(imgs, labels, 100)
    run = PersistentMLPRunner(tr, ep, steps_per_launch=550)
    res = {}
    for gap_ms in (0.0, 1.0, 5.0, 20.0):
        walls = []
        for rep in range(8):
            run.prepare(5)
            run.run(5, lookahead=20)
            torch.cuda.synchronize()
            assert run.error() == 0
            run.prepare(20)
            torch.cuda.synchronize()
            if gap_ms:
                time.sleep(gap_ms / 1e3)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run.run(20)
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e6)
        res[f"gap_{gap_ms}ms"] = [round(w, 1) for w in walls]
    # one stamped timed run: when do the copiers (next chunk over PCIe) finish vs the compute loop
    stamps = []
    for rep in range(4):
        run.prepare(5)
        run.run(5, lookahead=20)
        run.prepare(20)
        torch.cuda.synchronize()
        ts = torch.zeros(65 * 64 * 16, dtype=torch.int64, device=dev)
        run.phase_ts = ts
        run.run(20)
        torch.cuda.synchronize()
        run.phase_ts = None
        L = ts.cpu().numpy().reshape(65, 64, 16)[64].astype(np.float64) * 0.01
        t0 = min(L[:28, 0].min(), L[28:44, 0].min())
        stamps.append({"step0_start": round(float(ts.cpu().numpy().reshape(65, 64, 16)[0, :28, 0].max() * 0.01 - t0), 2),
                       "loop_done": round(float(L[:28, 3].max() - t0), 2),
                       "copier_done": round(float(L[28:44, 1].max() - t0), 2),
                       "copier_entry": round(float(L[28:44, 0].max() - t0), 2)})
    print(json.dumps({"bench_like_wall_us": res, "timed_run_launch_stamps_us": stamps}))


if __name__ == "__main__" and os.environ.get("BENCH_LIKE"):
    bench_like()
