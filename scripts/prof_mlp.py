"""Latency anatomy of the fused MLP step on one MI355X.

1. in-kernel phase timestamps (s_memrealtime, 10 ns ticks) for kernels A and B
2. graph-replayed per-launch cost of A alone, B alone, A+B, and a trivial kernel
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_example_amd.data.mnist import synthetic_mnist  # noqa: E402
from distributed_tensorflow_example_amd.models import mlp  # noqa: E402


def graph_time(fn, n=200, reps=5):
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    fn()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n):
            fn()
    out = []
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) * 1000.0 / n)
    return float(np.median(out))


def main():
    B = int(os.environ.get("B", "100"))
    dev = torch.device("cuda")
    tr = mlp.FusedMLPTrainer(batch_size=B, lr=0.0005, device=dev)
    C = tr.C
    imgs, labels = synthetic_mnist(B, seed=0)
    x = torch.from_numpy(imgs).to(dev).contiguous()
    y = torch.from_numpy(labels).to(dev).contiguous()
    tsA1 = torch.zeros(tr.nb * 7 * 2 * 16, dtype=torch.int64, device=dev)
    tsA2 = torch.zeros(tr.nb * 16, dtype=torch.int64, device=dev)
    tsB = torch.zeros(347 * 16, dtype=torch.int64, device=dev)

    def A1(ts=None):
        C.mlp_l1_fwd(x, 0, 0, B, tr.W1T, tr.z2p, ts)

    def A2(ts=None):
        C.mlp_head_bwd(tr.z2p, y, 0, B, tr.W2T, tr.W2N, tr.params, tr.dz2T, tr.partials, 1.0 / B, 0,
                       False, tr.gstep, ts)

    def A(ts=None):
        A1(None if ts is None else ts[0])
        A2(None if ts is None else ts[1])

    def Bk(ts=None):
        C.mlp_wgrad(x, 0, 0, tr.dz2T, B, tr.partials, tr.params, tr.W1T, tr.W2T, tr.W2N, None, 0,
                    tr.lr, tr.metrics, tr.gstep, ts)

    for _ in range(20):
        A()
        Bk()
    torch.cuda.synchronize()
    res = {}
    for it in range(3):
        A((tsA1, tsA2))
        Bk(tsB)
        torch.cuda.synchronize()
    T1 = tsA1.view(-1, 16).cpu().numpy()
    T2 = tsA2.view(-1, 16).cpu().numpy()
    TB = tsB.view(-1, 16).cpu().numpy()
    def phases(T, n):  # median per-phase durations (us) from consecutive stamps
        return [round(float(np.median(T[:, i + 1] - T[:, i])) / 100.0, 3) for i in range(n)]
    res["phases_us"] = {"A1": phases(T1, 3), "A2": phases(T2, 3), "B_strip": phases(TB[:343], 3)}
    last = {"A1": 3, "A2": 5, "B": 3}
    t1 = np.stack([T1[:, 0], T1[:, 3]], 1)
    t2 = np.stack([T2[:, 0], T2[:, 3]], 1)
    tb = np.stack([TB[:, 0], TB[:, 3]], 1)
    clk = lambda T, e: float(np.median((T[:, 8 + e] - T[:, 8]) / np.maximum(T[:, e] - T[:, 0], 1) * 100.0))
    res["core_clock_MHz"] = {"A1": clk(T1, 3), "A2": clk(T2, 3), "B": clk(TB[:343], 3)}
    base = t1[:, 0].min()
    f = lambda a: {"start_min": round((a[:, 0].min() - base) / 100.0, 2),
                   "start_max": round((a[:, 0].max() - base) / 100.0, 2),
                   "end_min": round((a[:, 1].min() - base) / 100.0, 2),
                   "end_max": round((a[:, 1].max() - base) / 100.0, 2),
                   "dur_med": round(float(np.median(a[:, 1] - a[:, 0])) / 100.0, 2)}
    res["A1"] = f(t1)
    res["A2"] = f(t2)
    res["B_strips"] = f(tb[:343])
    res["B_reducers"] = f(tb[343:])
    res["graph_us_per_launch"] = {
        "A1": graph_time(lambda: A1()),
        "A2": graph_time(lambda: A2()),
        "A": graph_time(lambda: A()),
        "B": graph_time(lambda: Bk()),
        "A+B": graph_time(lambda: (A(), Bk())),
        "apply_flat(trivial)": graph_time(lambda: C.mlp_apply_flat(tr.params, None, tr.lr, 0.0,
                                                                   tr.W1T, tr.W2T, tr.W2N)),
    }
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
