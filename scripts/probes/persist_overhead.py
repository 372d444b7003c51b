"""Fixed cost of one persistent-engine run (launch + prologue + epilogue +
Python) vs per-step cost: time run(n) for several n and fit t = a + b n.
Also the host-side cost of the run() call alone (no synchronize).

    python scripts/probes/persist_overhead.py [precision]
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
    torch.cuda.set_device(dev)
    imgs, labels = synthetic_mnist(55000, seed=0)
    tr = FusedMLPTrainer(batch_size=100, lr=0.0005, device=dev)
    ep = PinnedEpoch(imgs, labels, 100)
    run = PersistentMLPRunner(tr, ep, steps_per_launch=550, precision=prec)
    res = {}
    for n in (1, 2, 5, 10, 20, 50, 100, 200):
        ts, hs = [], []
        for rep in range(12):
            run.prepare(n)
            run.run(1, lookahead=n) if rep == 0 else None
            run.prepare(n)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run.run(n, lookahead=n)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            ts.append((t2 - t0) * 1e6)
            hs.append((t1 - t0) * 1e6)
        res[n] = (float(np.median(ts)), float(np.median(hs)))
    ns = np.array(sorted(res))
    t = np.array([res[k][0] for k in ns])
    b, a = np.polyfit(ns, t, 1)
    print(json.dumps({"precision": prec, "fit_fixed_us": round(a, 2), "fit_per_step_us": round(b, 3),
                      "median_us_by_steps": {int(k): round(res[k][0], 1) for k in ns},
                      "host_call_us_by_steps": {int(k): round(res[k][1], 1) for k in ns},
                      "copy_only_launches": run.copy_only_launches}))


if __name__ == "__main__":
    main()
