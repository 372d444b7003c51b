"""A/B of what sits inside bench.py's timed region around the persistent
run(20): with / without the timing event recorded before the launch, and
run() vs the bare prepared launch (Python planning cost).  Interleaved reps."""
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
    dev = torch.device("cuda", 0)
    imgs, labels = synthetic_mnist(55000, seed=0)
    tr = FusedMLPTrainer(batch_size=100, lr=0.0005, device=dev)
    ep = PinnedEpoch(imgs, labels, 100)
    run = PersistentMLPRunner(tr, ep, steps_per_launch=550)
    res = {"event+run": [], "run": [], "host_run_call": []}
    for rep in range(12):
        for variant in ("event+run", "run"):
            run.prepare(2)
            run.run(2, lookahead=20)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if variant == "event+run":
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
            run.run(20)
            th = time.perf_counter()
            torch.cuda.synchronize()
            res[variant].append((time.perf_counter() - t0) * 1e6)
            if variant == "run":
                res["host_run_call"].append((th - t0) * 1e6)
    print(json.dumps({k: round(float(np.median(v)), 1) for k, v in res.items()}))


if __name__ == "__main__":
    main()
