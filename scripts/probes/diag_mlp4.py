"""In-graph fork/join chunk prefetch vs serialized copy vs none."""
import json, os, sys
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
    C = tr.C
    stage = [torch.zeros(G * ep.rec, dtype=torch.uint8, device=dev) for _ in range(2)]

    def steps(buf):
        for i in range(G):
            off = i * ep.rec
            tr.enqueue_step(buf, off, 0, buf, off + B * 784)

    res = {}
    graphs = {}
    for mode in ("fork_join", "serial_copy", "none"):
        for par in (0, 1):
            steps(stage[par]); torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            cs = torch.cuda.Stream()
            side = torch.cuda.Stream()
            with torch.cuda.graph(g, stream=cs):
                m = torch.cuda.current_stream()
                if mode == "fork_join":
                    e0 = torch.cuda.Event(); e0.record(m)
                    side.wait_event(e0)
                    with torch.cuda.stream(side):
                        C.memcpy_h2d_async(stage[par ^ 1], 0, ep.host, 0, G * ep.rec)
                    e1 = torch.cuda.Event(); e1.record(side)
                    steps(stage[par])
                    m.wait_event(e1)
                elif mode == "serial_copy":
                    steps(stage[par])
                    C.memcpy_h2d_async(stage[par ^ 1], 0, ep.host, 0, G * ep.rec)
                else:
                    steps(stage[par])
            graphs[(mode, par)] = g
        def run(mode=mode):
            for j in range(NCH):
                graphs[(mode, j & 1)].replay()
        run(); torch.cuda.synchronize()
        res[mode] = gpu_time(run) / (G * NCH)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
