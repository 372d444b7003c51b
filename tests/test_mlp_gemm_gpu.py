"""Large-batch MLP step (csrc/kernels/mlp_gemm.hip + gemm.hip's exact-f32 MFMA
GEMM) vs the plain PyTorch fp32 reference step (models/mlp.py reference_step)."""
import numpy as np
import pytest
import torch

from distributed_tensorflow_example_amd.data.mnist import PinnedEpoch, synthetic_mnist
from distributed_tensorflow_example_amd.models import mlp

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B", [1024, 300, 4096])
@pytest.mark.parametrize("act", ["sigmoid", "relu"])
def test_gemm_step_matches_fp32_reference(native, B, act):
    imgs, labels = synthetic_mnist(B, seed=11)
    dev = torch.device("cuda")
    tr = mlp.GemmMLPTrainer(batch_size=B, lr=0.1, act=act, device=dev)
    p0 = tr.get_params().clone()
    tr.step_tensors(torch.from_numpy(imgs).to(dev), torch.from_numpy(labels).to(dev))
    torch.cuda.synchronize()
    loss, acc, g = mlp.reference_loss_and_grad(p0, torch.from_numpy(imgs).float() / 255.0,
                                               torch.from_numpy(labels), act)
    m = tr.read_metrics(0, 1)[0]
    assert abs(m[0] - loss.item()) < 1e-4 * max(1.0, abs(loss.item())), (m, loss)
    assert abs(m[1] - acc.item()) < 1e-6
    g_k = (p0 - tr.get_params()) / 0.1
    # fp32 operands end to end: only accumulation order differs
    for name, (off, shape) in mlp.PARAM_SPECS.items():
        n = int(np.prod(shape))
        a, b = g_k[off:off + n], g[off:off + n]
        err = (a - b).abs().max().item()
        assert err < 1e-4 * b.abs().max().item() + 1e-5, (name, err, b.abs().max().item())
    assert tr.global_step == 1


def test_gemm_runner_trains_and_matches_reference_run(native):
    """20 graph-replayed steps through MLPStepRunner (copy node + 7 launches per
    step) against 20 reference SGD steps on the same batches."""
    B, steps = 1024, 20
    imgs, labels = synthetic_mnist(B * 8, seed=4)
    dev = torch.device("cuda")
    tr = mlp.GemmMLPTrainer(batch_size=B, lr=0.0005, device=dev)
    flat = tr.get_params().clone()
    ep = PinnedEpoch(imgs, labels, B)
    run = mlp.MLPStepRunner(tr, ep, steps_per_graph=5)
    run.prepare(steps)
    run.run(steps)
    torch.cuda.synchronize()
    for s in range(steps):
        b = s % ep.num_batches
        x = torch.from_numpy(imgs[b * B:(b + 1) * B]).float() / 255.0
        y = torch.from_numpy(labels[b * B:(b + 1) * B])
        mlp.reference_step(flat, x, y, 0.0005)
    got = tr.get_params()
    rel = ((got - flat).norm() / flat.norm()).item()
    assert rel < 1e-5, rel
    m = tr.read_metrics(0, steps)
    assert np.all(np.isfinite(m)) and tr.global_step == steps


def test_gemm_engine_two_ranks_same_gpu(native):
    """bench.py's large-batch engine under torch.distributed.run with 2 ranks
    sharing cuda:0 (DTF_BENCH_SAME_GPU=1: gloo all-reduce of the flat fp32
    gradient between the slab reduce and the apply, eager launches): replicas
    must stay bit-identical (bench's consistency check) and one contract line
    comes out.  Timings are not multi-GPU numbers."""
    import json
    import os
    import socket
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(repo, "bench.py"), "--gpus", "2",
           "--batch", "512", "--steps", "10", "--warmup", "3", "--train-examples", "8192"]
    env = dict(os.environ, PYTHONPATH=repo, OMP_NUM_THREADS="2", DTF_BENCH_SAME_GPU="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=repo)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, (r.stdout + r.stderr)[-3000:]
    res = json.loads(lines[0])
    assert res["config"]["engine"] == "gemm" and res["config"]["parallelism"] == "dp2"
    assert res["global_steps_timed"] == 10 and res["value"] > 0
    assert res["config"]["global_batch"] == 1024
