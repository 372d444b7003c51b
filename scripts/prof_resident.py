"""Where the resident Session engine's per-run time goes (compat/resident.py,
ResidentMLPPlan; DTF_RESIDENT_STAMPS=1 turns on the kernel's per-run stamps).

The reference's loop body (example.py:164-171: train_op + cost + global_step
fetched with a fresh MNIST batch) runs `runs` times through the Session's
direct runner; for the last 64 runs the device stamps give (medians, us):
  door_to_copier    host door store -> copier 0 saw it (+ host memcpy before)  [host turnaround]
  copier_stage      copier 0: record rows over PCIe -> device stage
  handoff           copier 0 staged -> compute workgroup 0 saw all 14 copiers
  record_to_lds     the record from the stage into LDS / registers
  step              forward + head + backward + update
  write_through     variables written through to memory
  arrival           all 28 compute workgroups done
  publish           metrics + done count stored to pinned host memory
and the host's door -> done wait per run.  Prints one JSON line.

    DTF_RESIDENT_STAMPS=1 python scripts/prof_resident.py [runs]
"""
import json
import os
import sys
import time

import numpy as np

os.environ.setdefault("DTF_RESIDENT_STAMPS", "1")
os.environ.setdefault("DTF_RESIDENT_IDLE_S", "1.0")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

import torch  # noqa: E402


def main():
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.compat import lowering as L
    from distributed_tensorflow_example_amd.data.mnist import PixelBatch
    from test_lowering_cpu import _graph

    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 500
    rng = np.random.default_rng(0)
    B = 100
    pbs = [PixelBatch.of(u) for u in rng.integers(0, 256, (64, B, 784), dtype=np.uint8)]
    ys = np.eye(10, dtype=np.float32)[rng.integers(0, 10, (64, B))]
    g = _graph(tf)
    with tf.Session() as sess:
        sess.run(tf.global_variables_initializer())
        fetch = [g["train"], g["ce"], g["gs"]]
        for i in range(20):
            sess.run(fetch, feed_dict={g["x"]: pbs[i % 64], g["y_"]: ys[i % 64]})
        t0 = time.perf_counter()
        for i in range(runs):
            sess.run(fetch, feed_dict={g["x"]: pbs[i % 64], g["y_"]: ys[i % 64]})
        per_run = (time.perf_counter() - t0) / runs * 1e3
        rp = L.plan_for(g["train"])._rplan.plan
        st = rp.stamps()
        timing = rp.timing()
    if st is None:
        raise SystemExit("DTF_RESIDENT_STAMPS=1 is needed (set before the plan is built)")
    ts, wait = st[0].numpy().reshape(64, 8).astype(np.float64) * 0.01, st[1].numpy()   # 100 MHz -> us
    n_done = int(timing["runs"])
    order = [(n_done - 64 + k) % 64 for k in range(64)]     # oldest -> newest of the last 64 runs
    t = ts[order]
    names = ["copier_stage", "handoff", "record_to_lds", "step", "write_through", "arrival", "publish"]
    d = {nm: float(np.median(t[:, k + 1] - t[:, k])) for k, nm in enumerate(names)}
    d["door_to_copier_after_prev_publish"] = float(np.median(t[1:, 0] - t[:-1, 7]))
    d["device_run_total"] = float(np.median(t[:, 7] - t[:, 0]))
    out = {"session_run_ms": round(per_run, 4), "host_wait_us_median": round(float(np.median(wait)), 2),
           "stamps_us_median": {k: round(v, 2) for k, v in d.items()},
           "timing": {k: (round(v, 2) if isinstance(v, float) else v) for k, v in timing.items()}, "runs": runs}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
