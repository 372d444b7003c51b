"""The persistent weight-stationary MLP engine (csrc/kernels/mlp_persist_f32.hip:
exact-split bf16 MFMA "fp32" and f32-input MFMA "fp32-mfma") vs the plain
PyTorch fp32 reference of example.py's step (models/mlp.reference_step)."""
import numpy as np
import pytest
import torch

from distributed_tensorflow_example_amd.data.mnist import PinnedEpoch, synthetic_mnist
from distributed_tensorflow_example_amd.models import mlp

pytestmark = pytest.mark.gpu


def _ref_run(p0, imgs, labels, B, batches, lr, act="sigmoid"):
    """fp32 SGD over the given batch indices; returns params and per-step losses."""
    p = p0.clone()
    losses, accs = [], []
    for b in batches:
        x = torch.from_numpy(imgs[b * B:(b + 1) * B]).float() / 255.0
        y = torch.from_numpy(labels[b * B:(b + 1) * B])
        loss, acc = mlp.reference_step(p, x, y, lr, act)
        losses.append(loss.item())
        accs.append(acc.item())
    return p, np.array(losses), np.array(accs)


@pytest.mark.parametrize("engine", ["fp32", "fp32-mfma"])
@pytest.mark.parametrize("B", [100, 37, 112])
@pytest.mark.parametrize("act", ["sigmoid", "relu"])
def test_persist_f32_one_step_gradient_fp32_exact(native, B, act, engine):
    """fp32 engine: every parameter's gradient within 1e-5 (relative, per tensor)
    of the fp32 autograd reference.  lr = 1000 makes lr*g >> ulp(W), so the
    gradient recovered from the update is accurate to ~1e-8."""
    imgs, labels = synthetic_mnist(B, seed=11)
    dev = torch.device("cuda")
    lr = 1000.0
    tr = mlp.FusedMLPTrainer(batch_size=B, lr=lr, act=act, device=dev)
    p0 = tr.get_params().clone()
    ep = PinnedEpoch(imgs, labels, B)
    run = mlp.PersistentMLPRunner(tr, ep, steps_per_launch=1, precision=engine)
    run.run(1)
    torch.cuda.synchronize()
    assert run.error() == 0
    assert tr.global_step == 1
    x = torch.from_numpy(imgs).float() / 255.0
    loss, acc, g = mlp.reference_loss_and_grad(p0, x, torch.from_numpy(labels), act)
    g_k = (p0.double() - tr.get_params().double()) / lr
    for name, (off, shape) in mlp.PARAM_SPECS.items():
        n = int(np.prod(shape))
        a, b = g_k[off:off + n], g[off:off + n].double()
        rel = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
        assert rel < 1e-5, (name, rel)
    m = tr.read_metrics(0, 1)[0]
    assert abs(m[0] - loss.item()) < 1e-5 * max(1.0, abs(loss.item())), (m, loss)
    assert abs(m[1] - acc.item()) < 1e-6


@pytest.mark.parametrize("engine", ["fp32", "fp32-mfma"])
def test_persist_f32_multi_step_matches_reference(native, engine):
    """11 steps over wrapping chunks (cold start, in-kernel prefetch, offsets into
    a staged chunk, epoch wrap): fp32 engine tracks fp32 SGD to ~1e-6."""
    B, nb = 100, 6
    imgs, labels = synthetic_mnist(B * nb, seed=12)
    dev = torch.device("cuda")
    lr = 0.05
    tr = mlp.FusedMLPTrainer(batch_size=B, lr=lr, device=dev)
    p0 = tr.get_params().clone()
    ep = PinnedEpoch(imgs, labels, B)
    run = mlp.PersistentMLPRunner(tr, ep, steps_per_launch=4, precision=engine)
    run.run(7)     # (0,4) cold copy, (4,2), (0,1) epoch wrap; speculative (1,4) staged
    run.run(2)     # (1,2): inside the staged (1,4); streams (3,2) into the other stage
    run.run(2)     # (3,2): staged by the previous launch
    torch.cuda.synchronize()
    assert run.error() == 0
    assert tr.global_step == 11
    assert run.copy_only_launches == 1
    batches = [0, 1, 2, 3, 4, 5, 0, 1, 2, 3, 4]
    p_ref, losses, accs = _ref_run(p0, imgs, labels, B, batches, lr)
    d_k = tr.get_params().double() - p0.double()
    d_r = p_ref.double() - p0.double()
    rel = ((d_k - d_r).norm() / d_r.norm()).item()
    assert rel < 2e-5, rel
    m = tr.read_metrics(0, 11)
    assert np.allclose(m[:, 0], losses, rtol=1e-5, atol=1e-5), (m[:, 0], losses)
    assert np.allclose(m[:, 1], accs, atol=1e-6)


@pytest.mark.parametrize("precision", ["fp32", "fp32-mfma"])
def test_persist_short_timed_run_streams_only_what_it_computes(native, precision):
    """The bench's pattern: warmup(5) primes exactly the timed run's chunk; the
    timed run(20) needs no copy-only launch and prefetches <= 20 steps; the
    per-step device stamps give 20 positive durations."""
    B = 100
    imgs, labels = synthetic_mnist(B * 550, seed=15)
    dev = torch.device("cuda")
    tr = mlp.FusedMLPTrainer(batch_size=B, lr=0.0005, device=dev)
    ep = PinnedEpoch(imgs, labels, B)
    run = mlp.PersistentMLPRunner(tr, ep, steps_per_launch=550, precision=precision)
    run.prepare(5)
    run.run(5, lookahead=20)
    torch.cuda.synchronize()
    cold = run.copy_only_launches
    s0 = tr.global_step
    run.run(20)
    torch.cuda.synchronize()
    assert run.error() == 0
    assert run.copy_only_launches == cold
    assert 0 < run.last_prefetch_steps <= 20
    dt = run.step_times_ms(s0, s0 + 20)
    assert dt.shape == (20,) and (dt > 0).all() and (dt < 1.0).all(), dt


@pytest.mark.parametrize("precision", ["fp32", "fp32-mfma"])
def test_persist_deterministic_and_hands_over_to_step_path(native, precision):
    B = 100
    imgs, labels = synthetic_mnist(B * 4, seed=13)
    dev = torch.device("cuda")
    outs = []
    for _ in range(2):
        tr = mlp.FusedMLPTrainer(batch_size=B, lr=0.01, device=dev)
        ep = PinnedEpoch(imgs, labels, B)
        run = mlp.PersistentMLPRunner(tr, ep, steps_per_launch=3, precision=precision)
        run.run(5)
        torch.cuda.synchronize()
        outs.append(tr.get_params())
    assert torch.equal(outs[0], outs[1])       # bit-identical replays
    # the 3-kernel path continues from the persistent state (bf16 shadows refreshed)
    p5 = tr.get_params().clone()
    x = torch.from_numpy(imgs[:B]).to(dev)
    y = torch.from_numpy(labels[:B]).to(dev)
    tr.step_tensors(x, y)
    torch.cuda.synchronize()
    assert tr.global_step == 6
    _, _, g = mlp.reference_loss_and_grad(p5, torch.from_numpy(imgs[:B]).float() / 255.0,
                                          torch.from_numpy(labels[:B]))
    g_k = (p5 - tr.get_params()) / 0.01
    assert ((g_k - g).norm() / g.norm()).item() < 3e-2


@pytest.mark.parametrize("precision", ["fp32", "fp32-mfma"])
def test_persist_long_run_learns(native, precision):
    """1000 steps on synthetic MNIST: loss goes down."""
    B = 100
    imgs, labels = synthetic_mnist(B * 50, seed=14)
    dev = torch.device("cuda")
    tr = mlp.FusedMLPTrainer(batch_size=B, lr=0.05, device=dev)
    ep = PinnedEpoch(imgs, labels, B)
    run = mlp.PersistentMLPRunner(tr, ep, steps_per_launch=50, precision=precision)
    run.run(1000)
    torch.cuda.synchronize()
    assert run.error() == 0
    m = tr.read_metrics(0, 1000)
    assert np.isfinite(m).all()
    assert m[-50:, 0].mean() < 0.7 * m[:50, 0].mean(), (m[:50, 0].mean(), m[-50:, 0].mean())


@pytest.mark.parametrize("precision,grad,exchange", [("fp32", "bf16", "one-shot"), ("fp32", "fp32", "one-shot"),
                                                     ("fp32", "bf16", "two-shot"), ("fp32", "fp32", "two-shot"),
                                                     ("fp32-mfma", "bf16", "one-shot"), ("fp32-mfma", "fp32", "two-shot")])
@pytest.mark.parametrize("nproc", [2, 3])
def test_persist_multi_rank_same_gpu(native, nproc, precision, grad, exchange):
    _persist_selftest(nproc, precision, grad, exchange)


@pytest.mark.parametrize("exchange", ["one-shot", "two-shot"])
def test_persist_four_ranks_same_gpu(native, exchange):
    """4 ranks (the W = 4 chunking of the two-shot exchange: 8 waves over 4
    owners) sharing cuda:0 with the default fp32 engine and bf16 payload."""
    _persist_selftest(4, "fp32", "bf16", exchange)


@pytest.mark.parametrize("grad,exchange", [("bf16", "one-shot"), ("bf16", "two-shot"), ("fp32", "one-shot"),
                                           ("fp32", "two-shot")])
def test_persist_eight_ranks_same_gpu(native, grad, exchange):
    """W = 8 (the driver's whole-node N): the 8-wide peer table, 7 peers per
    workgroup and the two-shot chunking with one wave chunk per owner, with 8
    ranks sharing cuda:0.  Pre-staged input (no in-launch copiers), so the 8 x 28
    compute workgroups (224 of 256 CUs) can be co-resident."""
    _persist_selftest(8, "fp32", grad, exchange, prestaged=True, timeout=200)


@pytest.mark.parametrize("nproc", [5, 6])
def test_persist_five_six_ranks_same_gpu(native, nproc):
    """W between the unrolled peer-table widths (5, 6 -> the 8-wide table with
    absent entries) and two-shot chunks owned unevenly (w % W)."""
    _persist_selftest(nproc, "fp32", "bf16", "two-shot", prestaged=True, timeout=200)


def _persist_selftest(nproc, precision, grad, exchange, prestaged=False, timeout=100):
    """N ranks sharing cuda:0: in-kernel IPC exchange, bit-identical replicas, sync-SGD math."""
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
    cmd = [sys.executable, "-m", "torch.distributed.run", f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1",
           f"--master-port={port}", os.path.join(repo, "scripts", "persist_selftest.py"), "--same-gpu",
           "--steps=10", "--per-launch=4", f"--precision={precision}", f"--grad-dtype={grad}",
           f"--exchange={exchange}"] + (["--prestaged"] if prestaged else [])
    env = dict(os.environ, PYTHONPATH=repo, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    out = r.stdout + r.stderr
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and line, out[-3000:]
    res = json.loads(line[-1])
    assert res["persist_selftest"] == "pass", res


def test_bench_two_ranks_same_gpu_short_run(native):
    """bench.py as the driver launches it for N=2 (torch.distributed.run, one
    rank per 'GPU'), at the driver's short step count, with both ranks sharing
    cuda:0 (DTF_BENCH_SAME_GPU=1: gloo control plane, IPC data plane): the
    exchange strategy is chosen and validated, the timed run completes, and
    rank 0 prints one contract JSON line.  Timings are not multi-GPU numbers."""
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
           "--steps", "20", "--warmup", "5", "--tune-steps", "40"]
    env = dict(os.environ, PYTHONPATH=repo, OMP_NUM_THREADS="2", DTF_BENCH_SAME_GPU="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=repo)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, (r.stdout + r.stderr)[-3000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["steps"] == 20 and res["warmup"] == 5
    assert res["value"] > 0 and res["ms_per_step"] > 0 and res["dtype"] == "fp32"
    assert res["config"]["parallelism"] == "dp2"


def test_bench_two_ranks_timed_run_fault_falls_back(native):
    """A failure inside the timed run does not lose the scaling point: rank 1
    stops publishing its exchange flag from timed step 5 on (a dead peer) (DTF_BENCH_FAULT -> the kernel's
    mlpf_set_fault), its peer times out, the replica check fails, and bench.py
    re-times the next validated strategy in the same process and prints one
    contract line naming the failed mode under `fallbacks`."""
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
           "--steps", "20", "--warmup", "5", "--tune-steps", "40", "--exchange-timeout", "2"]
    env = dict(os.environ, PYTHONPATH=repo, OMP_NUM_THREADS="2", DTF_BENCH_SAME_GPU="1", DTF_BENCH_FAULT="5")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=repo)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, (r.stdout + r.stderr)[-3000:]
    res = json.loads(lines[0])
    fb = res["config"]["fallbacks"] or {}
    failed = [m for m, why in fb.items() if "timed run" in why]
    assert len(failed) == 1, (fb, r.stderr[-4000:])
    assert res["config"]["exchange_mode"] != failed[0]
    assert res["value"] > 0 and res["steps"] == 20 and res["n_gpus"] == 2
    assert res["global_steps_timed"] == 20


def _bench_plain(n, extra_env=None, extra_args=(), timeout=150):
    """`python bench.py --gpus n` as ONE plain process (no torchrun): bench.py
    starts the n rank processes itself; all share cuda:0 (DTF_BENCH_SAME_GPU)."""
    import json
    import os
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(PYTHONPATH=repo, OMP_NUM_THREADS="2", DTF_BENCH_SAME_GPU="1", **(extra_env or {}))
    cmd = [sys.executable, os.path.join(repo, "bench.py"), "--gpus", str(n), "--steps", "20", "--warmup", "5",
           "--tune-steps", "40"] + list(extra_args)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=repo)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, (r.stdout + r.stderr)[-3000:]
    return json.loads(lines[0]), r


@pytest.mark.parametrize("n", [2, 4])
def test_bench_self_launch_without_torchrun(native, n):
    """The verdict's launch-shape item: `bench.py --gpus N` without
    torch.distributed.run prints exactly one contract line for the N-rank job."""
    res, _ = _bench_plain(n)
    assert res["n_gpus"] == n and res["steps"] == 20 and res["warmup"] == 5
    assert res["config"]["parallelism"] == f"dp{n}" and res["config"]["global_batch"] == 100 * n
    assert res["config"]["launch"] == "self-launched rank processes"
    assert res["config"]["exchange_mode"].startswith("persistent")
    assert res["value"] > 0


def test_bench_rccl_init_failure_still_measures(native):
    """RCCL that cannot come up (injected init fault) costs only the RCCL
    strategy: it is tried first here (DTF_BENCH_CHAIN), recorded under
    `fallbacks`, and the in-kernel exchange still produces the line."""
    res, r = _bench_plain(2, {"DTF_FAULT_RCCL_INIT": "1", "DTF_BENCH_CHAIN": "rccl,persistent"})
    fb = res["config"]["fallbacks"] or {}
    assert "rccl" in fb and "fault injected" in fb["rccl"], (fb, r.stderr[-3000:])
    assert res["config"]["exchange_mode"] == "persistent" and res["value"] > 0
    assert "fault injected" in (res["config"]["rccl_comm"] or "")
