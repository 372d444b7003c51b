"""Isolate what separates the bench step time from the tight-graph step time.

(a) graph of G steps, every step reads the SAME batch (L2-hot x)
(b) graph of G steps over G different batches already resident on device
(c) (b) + a concurrent chunk hipMemcpyAsync on a side stream (the bench's pipeline)
(d) the MLPStepRunner itself
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_example_amd.data.mnist import PinnedEpoch, synthetic_mnist  # noqa: E402
from distributed_tensorflow_example_amd.models import mlp  # noqa: E402


def timeit(fn, reps=20):
    out = []
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) * 1000.0)
    return float(np.median(out))


def main():
    B, G = 100, 50
    dev = torch.device("cuda")
    imgs, labels = synthetic_mnist(55000, seed=1)
    ep = PinnedEpoch(imgs, labels, B)
    tr = mlp.FusedMLPTrainer(batch_size=B, lr=0.0005, device=dev)
    stage = torch.zeros(G * ep.rec, dtype=torch.uint8, device=dev)
    stage2 = torch.zeros(G * ep.rec, dtype=torch.uint8, device=dev)
    tr.C.memcpy_h2d_async(stage, 0, ep.host, 0, G * ep.rec)
    torch.cuda.synchronize()
    res = {}

    def mk(same):
        def f():
            for i in range(G):
                off = 0 if same else i * ep.rec
                tr.enqueue_step(stage, off, 0, stage, off + B * 784)
        return f

    graphs = {}
    for name, same in (("a_same_x", True), ("b_diff_x", False)):
        f = mk(same)
        f()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        with torch.cuda.graph(g, stream=s):
            f()
        graphs[name] = g
        res[name + "_us_per_step"] = timeit(g.replay) / G
    side = torch.cuda.Stream()

    def with_copy():
        ev = torch.cuda.Event()
        ev.record()
        side.wait_event(ev)
        with torch.cuda.stream(side):
            tr.C.memcpy_h2d_async(stage2, 0, ep.host, G * ep.rec, G * ep.rec)
        graphs["b_diff_x"].replay()
        torch.cuda.current_stream().wait_stream(side)

    res["c_diff_x_concurrent_copy_us_per_step"] = timeit(with_copy) / G
    res["copy_alone_us_per_chunk"] = timeit(
        lambda: tr.C.memcpy_h2d_async(stage2, 0, ep.host, G * ep.rec, G * ep.rec))
    r = mlp.MLPStepRunner(tr, ep, steps_per_graph=G)
    r.prepare(G * 20)
    r.run(G * 4)
    torch.cuda.synchronize()
    res["d_runner_us_per_step"] = timeit(lambda: r.run(G * 4), reps=5) / (G * 4)
    r2 = mlp.MLPStepRunner(tr, ep, steps_per_graph=110)
    r2.prepare(550)
    r2.run(550)
    torch.cuda.synchronize()
    res["d_runner_g110_us_per_step"] = timeit(lambda: r2.run(550), reps=3) / 550
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
