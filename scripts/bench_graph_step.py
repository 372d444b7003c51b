"""Per-step cost of the compat graph path (examples/mnist_example.py's graph,
no --fused): Session.run wall time per step on the resident engine (MNIST
loader batches, compat/resident.py), on the launched lowered kernels
(DTF_RESIDENT_SESSION=0; loader batches and plain float32 feeds) and on the
eager op-by-op path (DTF_GRAPH_LOWERING=0), plus device time of the lowered
kernels alone (CUDA events around graph_mlp_step).

    python scripts/bench_graph_step.py [steps]
    python scripts/bench_graph_step.py --workers 2 [steps]   # 1 ps + 2 sync workers (IPC plane)
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main_workers(workers: int, steps: int):
    """examples/mnist_example.py as 1 ps + `workers` synchronous workers (all on
    the visible GPU(s); on a 1-GPU box they share cuda:0 -- a rehearsal of the
    protocol, not a scaling number): per-Session.run time of the reference's
    loop past its first 20 runs, per worker, with the data-plane facts."""
    import tempfile

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
    from test_compat_ipc_gpu import run_cluster

    with tempfile.TemporaryDirectory() as tmp:
        _, facts, _ = run_cluster(tmp, workers, steps, extra=["--train_size=20000"], timeout=600)
    ms = [f["session_loop_ms_per_step_after_20"] for f in facts]
    print(json.dumps({"workers": workers, "steps": steps,
                      "session_run_ms_per_step_workers": [round(m, 4) for m in ms],
                      "session_run_ms_per_step_max": round(max(ms), 4),
                      "native_plan_ipc": all(f["native_plan_ipc"] for f in facts),
                      "native_plan_steps": [f["native_plan_steps"] for f in facts],
                      "rccl_comm": any(f["rccl_comm"] for f in facts),
                      "ipc_calls": [f["ipc_calls"] for f in facts],
                      "same_gpu": torch.cuda.device_count() < workers}))


def main():
    if "--workers" in sys.argv:
        i = sys.argv.index("--workers")
        workers = int(sys.argv[i + 1])
        rest = [a for j, a in enumerate(sys.argv[1:], 1) if j not in (i, i + 1)]
        return main_workers(workers, int(rest[0]) if rest else 1000)
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd import _native
    from distributed_tensorflow_example_amd.compat import lowering as L
    from test_lowering_cpu import _graph

    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    rng = np.random.default_rng(0)
    B = 100
    from distributed_tensorflow_example_amd.data.mnist import PixelBatch

    u8s = rng.integers(0, 256, (64, B, 784), dtype=np.uint8)
    pbs = [PixelBatch.of(u) for u in u8s]           # what the MNIST loader's next_batch returns
    xs = np.stack([np.asarray(p) for p in pbs])     # the same values as plain float32 arrays
    ys = np.eye(10, dtype=np.float32)[rng.integers(0, 10, (64, B))]
    out = {}
    from distributed_tensorflow_example_amd.compat import resident as R

    for mode in ("resident", "u8", "1", "0"):
        os.environ["DTF_GRAPH_LOWERING"] = "0" if mode == "0" else "1"
        os.environ["DTF_RESIDENT_SESSION"] = "1" if mode == "resident" else "0"
        feeds = pbs if mode in ("resident", "u8") else xs
        g = _graph(tf)
        with tf.Session() as sess:
            sess.run(tf.global_variables_initializer())
            fetch = [g["train"], g["ce"], g["gs"]]
            for i in range(20):
                sess.run(fetch, feed_dict={g["x"]: feeds[i % 64], g["y_"]: ys[i % 64]})
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(steps):
                sess.run(fetch, feed_dict={g["x"]: feeds[i % 64], g["y_"]: ys[i % 64]})
            torch.cuda.synchronize()
            out[{"resident": "resident", "u8": "lowered_u8", "1": "lowered", "0": "eager"}[mode]] = \
                (time.perf_counter() - t0) / steps * 1e3
            if mode == "resident":
                plan = L.plan_for(g["train"])
                out["resident_steps"] = int(plan.resident_steps)
                rp = plan._rplan.plan
                out["resident_split_us"] = {k: round(v, 2) if isinstance(v, float) else v
                                            for k, v in rp.timing().items()}
                R.quiesce_all()
            if mode == "u8":
                cp = L.plan_for(g["train"])._cplan
                t0 = time.perf_counter()
                for i in range(1000):
                    cp.run_u8(u8s[i % 64], ys[i % 64], 0.0, True)
                out["native_call_u8_us"] = (time.perf_counter() - t0) / 1000 * 1e6
                out["native_call_u8_split_us"] = {k: round(v, 2) if isinstance(v, float) else v
                                                  for k, v in cp.timing().items()}
            if mode == "1":
                plan = L.plan_for(g["train"])
                assert plan is not None and plan.steps >= steps
                # device time of the three kernels alone
                C = _native.load()
                W1, b1, W2, b2 = (v.value.data for v in (plan.pat.W1, plan.pat.b1, plan.pat.W2, plan.pat.b2))
                x = torch.from_numpy(xs[0]).cuda()
                y = torch.from_numpy(ys[0]).cuda()
                a2 = torch.empty(112 * 112, device="cuda")
                dz2 = torch.empty(112 * 112, device="cuda")
                met = torch.zeros(4, device="cuda")
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                for _ in range(10):
                    C.graph_mlp_step(x, y, W1, b1, W2, b2, a2, dz2, None, met, None, 0.0, 0, True, True)
                e0.record()
                for _ in range(1000):
                    C.graph_mlp_step(x, y, W1, b1, W2, b2, a2, dz2, None, met, None, 0.0, 0, True, True)
                e1.record()
                torch.cuda.synchronize()
                out["kernels_us"] = e0.elapsed_time(e1)     # the 3 kernels + the lr fill, back to back
                out["native_plan_runs"] = int(plan._cplan.steps())
                out["native_plan_hipgraph"] = bool(plan._cplan.use_graph())
                # the native call alone (feed packing + copy + kernels + metrics + sync), no Session
                cp = plan._cplan
                t0 = time.perf_counter()
                for i in range(1000):
                    cp.run(xs[i % 64], ys[i % 64], 0.0, True)
                out["native_call_us"] = (time.perf_counter() - t0) / 1000 * 1e6
                if hasattr(cp, "timing"):
                    out["native_call_split_us"] = {k: round(v, 2) if isinstance(v, float) else v
                                                   for k, v in cp.timing().items()}
        tf.reset_default_graph()
    os.environ.pop("DTF_GRAPH_LOWERING", None)
    os.environ.pop("DTF_RESIDENT_SESSION", None)
    print(json.dumps({"session_run_ms_per_step_resident_loader_batches": round(out["resident"], 4),
                      "resident_steps": out.get("resident_steps"),
                      "resident_split_us": out.get("resident_split_us"),
                      "native_plan_runs": out.get("native_plan_runs"),
                      "native_plan_hipgraph": out.get("native_plan_hipgraph"),
                      "native_call_us": round(out.get("native_call_us", 0.0), 2),
                      "native_call_split_us": out.get("native_call_split_us"),
                      "native_call_u8_us": round(out.get("native_call_u8_us", 0.0), 2),
                      "native_call_u8_split_us": out.get("native_call_u8_split_us"),
                      "session_run_ms_per_step_lowered_loader_batches": round(out["lowered_u8"], 4),
                      "session_run_ms_per_step_lowered": round(out["lowered"], 4),
                      "session_run_ms_per_step_eager": round(out["eager"], 4),
                      "lowered_kernels_us_per_step": round(out["kernels_us"], 3), "batch": B, "steps": steps}))


if __name__ == "__main__":
    main()
