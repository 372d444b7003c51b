"""Host-side cost of the headline's timed launch, piece by piece (us per call,
mean of back-to-back calls, nothing synchronised in between):
  pybind_noop      a trivial native call (mlpf_stage_rec)
  tiny_launch      a one-block native kernel launch (zero-fill of 16 floats via gemm's zero kernel path)
  plan_launch      PersistF32Plan.launch of a 1-step chunk (the engine's kernel, ~200 B of kernargs)
  runner_run       PersistentMLPRunner.run(1) (Python fast path + the same launch)
One JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_tensorflow_example_amd.data.mnist import PinnedEpoch, synthetic_mnist  # noqa: E402
from distributed_tensorflow_example_amd.models import mlp  # noqa: E402


def per_call(fn, n):
    t = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t) / n * 1e6


dev = torch.device("cuda", 0)
C = mlp._native.load()
imgs, labels = synthetic_mnist(55000, seed=1)
ep = PinnedEpoch(imgs, labels, 100)
tr = mlp.FusedMLPTrainer(batch_size=100, device=dev)
run = mlp.PersistentMLPRunner(tr, ep, steps_per_launch=550)
run.prepare(550)
run.run(550)
torch.cuda.synchronize()
out = {}
out["pybind_noop_us"] = round(per_call(lambda: C.mlpf_stage_rec(), 2000), 3)
a = torch.zeros(16, 16, device=dev)
b = torch.zeros(16, 16, device=dev)
o = torch.zeros(16, 16, device=dev)
torch.cuda.synchronize()
out["tiny_launch_us"] = round(per_call(lambda: C.gemm(a, False, b, False, o, None, 0, 1.0, 0.0, None), 200), 3)
torch.cuda.synchronize()
st = run.staged[0]
out["plan_launch_us"] = round(per_call(lambda: run._plan.launch(0, 0, 1, 0, 0), 100), 3)
torch.cuda.synchronize()
run.cursor = st[0] if st else 0
out["runner_run_us"] = round(per_call(lambda: run.run(1, lookahead=0), 100), 3)
torch.cuda.synchronize()
# the timed-region shape: sync, then one launch after an idle host
vals = []
for _ in range(50):
    torch.cuda.synchronize()
    t = time.perf_counter()
    run._plan.launch(0, 0, 1, 0, 0)
    vals.append((time.perf_counter() - t) * 1e6)
torch.cuda.synchronize()
vals.sort()
out["plan_launch_after_sync_p50_us"] = round(vals[len(vals) // 2], 3)
print(json.dumps(out), flush=True)
