"""Runner prefetch variants: where does the chunk copy overlap the replay?"""
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_example_amd.data.mnist import PinnedEpoch, synthetic_mnist  # noqa
from distributed_tensorflow_example_amd.models import mlp  # noqa


def timeit(fn, reps=5):
    out = []
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) * 1000.0)
    return float(np.median(out))


def main():
    B, G = 100, 50
    dev = torch.device("cuda")
    imgs, labels = synthetic_mnist(55000, seed=1)
    ep = PinnedEpoch(imgs, labels, B)
    tr = mlp.FusedMLPTrainer(batch_size=B, lr=0.0005, device=dev)
    res = {}
    for name, prio in (("side_prio0", 0), ("side_prio_high", -1)):
        r = mlp.MLPStepRunner(tr, ep, steps_per_graph=G)
        r.prepare(G * 12)
        r.side = torch.cuda.Stream(device=dev, priority=prio)  # created after capture streams
        r.run(G * 4); torch.cuda.synchronize()
        res[name] = timeit(lambda: r.run(G * 8)) / (G * 8)
    # copy on a non-default main stream
    r = mlp.MLPStepRunner(tr, ep, steps_per_graph=G)
    r.prepare(G * 12)
    ms = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(ms):
        r.run(G * 4)
    torch.cuda.synchronize()
    def f():
        with torch.cuda.stream(ms):
            r.run(G * 8)
        torch.cuda.current_stream().wait_stream(ms)
    res["main_nondefault_stream"] = timeit(f) / (G * 8)
    # no prefetch at all (data already staged; measures pure replay chain)
    r = mlp.MLPStepRunner(tr, ep, steps_per_graph=G)
    r.prepare(G * 2)
    g = r._graph(G, 0)
    res["replay_only"] = timeit(lambda: [g.replay() for _ in range(8)]) / (G * 8)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
