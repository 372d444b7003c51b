"""Does anything else in the process make the resident Session engine exit
between runs?  Runs example.py's graph on the resident engine for 6 steps
(with the W-parameter reads the GPU tests do between runs) after an optional
preamble, and prints launches / step times / the engine's stream kind.

    python scripts/probes/resident_relaunch.py [none|world|streams|sparse]
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    os.environ["DTF_RESIDENT_IDLE_S"] = "2.0"
    pre = sys.argv[1] if len(sys.argv) > 1 else "none"
    from test_lowering_cpu import _graph
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.compat import lowering as L
    from distributed_tensorflow_example_amd.data.mnist import PixelBatch

    keep = []
    if pre == "world":
        from distributed_tensorflow_example_amd.parallel import world as W
        keep.append(W.init())
    elif pre == "streams":
        keep += [torch.cuda.Stream() for _ in range(8)]
        for s in keep:
            with torch.cuda.stream(s):
                torch.ones(10, device="cuda").sum()
        torch.cuda.synchronize()
    elif pre == "sparse":
        from distributed_tensorflow_example_amd.models.sparse_lr import SparseLRTrainer
        from distributed_tensorflow_example_amd.parallel import world as W
        w = W.init()
        tr = SparseLRTrainer(100000, 0.5, w, seed=1)
        offs = np.arange(0, 65, 8, dtype=np.int64)
        tr.train_step((np.zeros((8, 1), np.float32), offs, np.arange(64, dtype=np.int64), np.ones(64, np.float32)))
        torch.cuda.synchronize()
        keep += [w, tr]
    g = _graph(tf)
    rng = np.random.default_rng(0)
    out = {"preamble": pre, "step_ms": []}
    with tf.Session() as sess:
        sess.run(tf.global_variables_initializer())
        for s in range(6):
            bx = PixelBatch.of(rng.integers(0, 256, (100, 784), dtype=np.uint8))
            by = np.eye(10, dtype=np.float32)[rng.integers(0, 10, 100)]
            t0 = time.perf_counter()
            sess.run([g["train"], g["ce"]], feed_dict={g["x"]: bx, g["y_"]: by})
            out["step_ms"].append(round((time.perf_counter() - t0) * 1e3, 2))
            t1 = time.perf_counter()
            [v.numpy() for v in g["W"]]
            out.setdefault("read_ms", []).append(round((time.perf_counter() - t1) * 1e3, 2))
        plan = L.plan_for(g["train"])
        rp = getattr(plan, "_rplan", None)
        out["resident_steps"] = getattr(plan, "resident_steps", 0)
        if rp is not None:
            out["timing"] = {k: v for k, v in rp.plan.timing().items()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
