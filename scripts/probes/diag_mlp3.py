"""Host-side timing of the runner loop pieces + variants."""
import json, os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_example_amd.data.mnist import PinnedEpoch, synthetic_mnist  # noqa
from distributed_tensorflow_example_amd.models import mlp  # noqa


def gpu_time(fn):
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record(); fn(); e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0


def main():
    B, G, NCH = 100, 50, 8
    dev = torch.device("cuda")
    imgs, labels = synthetic_mnist(55000, seed=1)
    ep = PinnedEpoch(imgs, labels, B)
    tr = mlp.FusedMLPTrainer(batch_size=B, lr=0.0005, device=dev)
    r = mlp.MLPStepRunner(tr, ep, steps_per_graph=G)
    r.prepare(G * 20)
    g0, g1 = r._graph(G, 0), r._graph(G, 1)
    C = tr.C
    side = r.side
    main = torch.cuda.current_stream()
    res = {}
    host = {"replay": [], "copy": [], "events": []}

    def variant(kind):
        freed = None
        for j in range(NCH):
            par = j & 1
            t0 = time.perf_counter()
            (g0 if par == 0 else g1).replay()
            t1 = time.perf_counter()
            if kind == "none":
                continue
            if kind == "main_copy":
                C.memcpy_h2d_async(r.stage[par ^ 1], 0, ep.host, 0, G * ep.rec)
                continue
            evc = torch.cuda.Event()
            if freed is not None:
                side.wait_event(freed)
            t2 = time.perf_counter()
            if kind == "side_copy":
                with torch.cuda.stream(side):
                    C.memcpy_h2d_async(r.stage[par ^ 1], 0, ep.host, 0, G * ep.rec)
            t3 = time.perf_counter()
            evc.record(side)
            freed = torch.cuda.Event()
            freed.record(main)
            main.wait_event(evc)
            t4 = time.perf_counter()
            if kind == "side_copy":
                host["replay"].append((t1 - t0) * 1e6)
                host["copy"].append((t3 - t2) * 1e6)
                host["events"].append((t4 - t3 + t2 - t1) * 1e6)

    for kind in ("none", "events_only", "side_copy", "main_copy"):
        variant(kind)
        torch.cuda.synchronize()
        res[kind] = gpu_time(lambda: variant(kind)) / (G * NCH)
    res["host_us"] = {k: float(np.median(v)) for k, v in host.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
