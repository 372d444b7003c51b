"""Model-level GPU tests: sparse LR on the HIP embedding-bag / sigmoid-xent /
scatter-SGD kernels vs an fp64 reference, the compat MLP graph, and the
example programs on cuda:0 (single-worker cluster)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sparse_lr_step_matches_fp64_reference(native, tmp_path):
    from distributed_tensorflow_example_amd.data import libsvm
    from distributed_tensorflow_example_amd.models import sparse_lr
    from distributed_tensorflow_example_amd.parallel.world import World

    files = libsvm.write_synthetic(str(tmp_path / "p"), 1, 1500, 50000, 20, seed=3)
    data = libsvm.load_files(files)
    w = World(device=torch.device("cuda", 0))
    tr = sparse_lr.SparseLRTrainer(50000, 0.3, w, seed=2)
    assert tr.W.local.is_cuda
    for s in range(3):
        b = data.slice(s * 500, (s + 1) * 500)
        W0, b0 = tr.W.local.detach().cpu().clone(), tr.b.detach().cpu().clone()
        lab, off, ids, vals = [torch.from_numpy(x) for x in (b.labels, b.offsets, b.ids, b.vals)]
        l_ref, gW, gb = sparse_lr.reference_loss_grad(W0, b0, lab, off, ids, vals)
        loss = tr.train_step(b)
        assert abs(float(loss) - float(l_ref)) < 1e-4
        assert torch.allclose(tr.W.local.cpu(), (W0.double() - 0.3 * gW).float(), atol=2e-5)
        assert torch.allclose(tr.b.detach().cpu(), (b0.double() - 0.3 * gb).float(), atol=1e-5)
    tr.reset_auc()
    tr.auc_update(data.slice(0, 1500))
    a = tr.auc()
    assert 0.0 <= a <= 1.0


def test_sharded_embedding_bag_dim128_on_gpu(native):
    from distributed_tensorflow_example_amd.parallel.sharded_embedding import ShardedEmbedding
    from distributed_tensorflow_example_amd.parallel.world import World

    w = World(device=torch.device("cuda", 0))
    emb = ShardedEmbedding(100000, 128, w, init_std=0.1, seed=1)
    ids = torch.randint(0, 100000, (3000,), device="cuda")
    offs = torch.arange(0, 3001, 30, device="cuda")
    full = emb.local.detach().cpu().clone()
    out, st = emb.bag_forward(ids, offs, None, "mean")
    ref = torch.nn.functional.embedding_bag(ids.cpu(), full, offs[:-1].cpu(), mode="mean")
    assert torch.allclose(out.cpu(), ref, atol=1e-5)
    out.sum().backward()
    emb.bag_backward_sgd(st, 1.0)
    Wr = full.clone().requires_grad_()
    torch.nn.functional.embedding_bag(ids.cpu(), Wr, offs[:-1].cpu(), mode="mean").sum().backward()
    assert torch.allclose(emb.local.cpu(), full - Wr.grad, atol=1e-5)


def test_mnist_example_single_worker_gpu(tmp_path):
    for fused in ("--nofused", "--fused", "--fused --persistent"):
        p = _free_port()
        env = dict(os.environ, PYTHONPATH=REPO)
        cmd = [sys.executable, os.path.join(REPO, "examples", "mnist_example.py"), "--job_name=worker",
               "--task_index=0", "--ps_hosts=", f"--worker_hosts=127.0.0.1:{p}", "--max_steps=300",
               "--train_size=10000", "--learning_rate=0.1", f"--logs_path={tmp_path}/logs",
               f"--result_json={tmp_path}/r.json"] + fused.split()
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stdout + r.stderr
        res = json.load(open(tmp_path / "r.json"))
        assert res["global_step"] == 300
        assert res["accuracy"] > 0.5, res


def test_sparse_lr_graphed_step_matches_eager(monkeypatch):
    """The device-resident sparse LR step captured in one hipGraph
    (utils/graphs.GraphedStep) trains like the launch-by-launch step:
    capture warmups leave no trace, replays see the new batches.  (The
    general sharded path: one worker otherwise takes the fused kernels.)"""
    import numpy as np

    monkeypatch.setenv("DTF_SLR_FUSED", "0")

    from distributed_tensorflow_example_amd.models.sparse_lr import SparseLRTrainer
    from distributed_tensorflow_example_amd.parallel import world as W

    w = W.get_world() if W._WORLD is not None else W.init()
    rng = np.random.default_rng(0)
    B, nnz, F = 500, 40, 1_000_000
    batches = []
    for _ in range(6):
        ids = torch.from_numpy(((rng.zipf(1.1, B * nnz) - 1) % F).astype(np.int64)).cuda()
        offs = torch.arange(0, B * nnz + 1, nnz, dtype=torch.int64, device="cuda")
        vals = torch.rand(B * nnz, device="cuda")
        lab = (torch.rand(B, 1, device="cuda") < 0.3).float()
        batches.append((lab, offs, ids, vals))
    eager = SparseLRTrainer(F, 1.0, w, seed=3)
    graphed = SparseLRTrainer(F, 1.0, w, seed=3)
    graphed.enable_graph()
    for i in range(12):
        le = eager.train_step(batches[i % 6])
        lg = graphed.train_step(batches[i % 6])
        assert abs(float(le) - float(lg)) < 1e-5, i
    assert graphed._graphed.captures == 1 and graphed._graphed.replays == 12
    assert graphed.global_step == eager.global_step == 12
    assert torch.allclose(eager.W.local, graphed.W.local, atol=1e-5)
    assert torch.allclose(eager.b, graphed.b, atol=1e-6)


def test_wide_deep_graphed_step_matches_eager(native):
    """The whole W&D step (routing, lookups, bags, MFMA tower, loss, backward,
    sparse SGD of both tables, fused Adam) replayed as one hipGraph follows the
    eager step."""
    from distributed_tensorflow_example_amd.models.wide_deep import WideDeep
    from distributed_tensorflow_example_amd.parallel import world as W

    w = W.get_world() if W._WORLD is not None else W.init()
    F, B, nnz = 50_000, 256, 8
    g = torch.Generator(device="cuda").manual_seed(0)
    batches = []
    for _ in range(5):
        ids = torch.randint(0, F, (B * nnz,), device="cuda", generator=g)
        offs = torch.arange(0, B * nnz + 1, nnz, device="cuda")
        vals = torch.rand(B * nnz, device="cuda", generator=g)
        lab = (torch.rand(B, 1, device="cuda", generator=g) < 0.3).float()
        batches.append((lab, offs, ids, vals))
    mk = lambda: WideDeep(F, emb_dim=16, hidden=(64, 32), lr=0.5, dense_opt="adam", dense_lr=0.01, world=w,
                          seed=4, ids_capacity=B * nnz)
    eager, graphed = mk(), mk()
    graphed.enable_graph()
    for i in range(10):
        le = eager.train_step(batches[i % 5])
        lg = graphed.train_step(batches[i % 5])
        assert abs(float(le) - float(lg)) < 1e-4, (i, float(le), float(lg))
    assert graphed._graphed.captures == 1 and graphed._graphed.replays == 10
    assert graphed.global_step == eager.global_step == 10
    assert torch.allclose(eager.emb.local, graphed.emb.local, atol=1e-5)
    assert torch.allclose(eager.wide.local, graphed.wide.local, atol=1e-5)
    for a, b in zip(eager.dense_params, graphed.dense_params):
        assert torch.allclose(a, b, atol=1e-5)


def test_wide_deep_gpu_step_matches_cpu_reference(native):
    """The GPU step -- fused head (wide + tower + bias, xent, mean: one kernel
    forward, one backward), tower weight / bias gradients accumulated straight
    into the flat gradient bucket, sparse SGD of both tables, fused Adam --
    against the same model on the CPU (plain torch autograd and ops), same
    Philox / generator initialisation, 4 steps."""
    from distributed_tensorflow_example_amd.models.wide_deep import WideDeep
    from distributed_tensorflow_example_amd.parallel.world import World

    F, B, nnz = 20_000, 128, 6
    gen = torch.Generator().manual_seed(7)
    batches = []
    for _ in range(4):
        ids = torch.randint(0, F, (B * nnz,), generator=gen)
        offs = torch.arange(0, B * nnz + 1, nnz)
        vals = torch.rand(B * nnz, generator=gen)
        lab = (torch.rand(B, 1, generator=gen) < 0.3).float()
        batches.append((lab, offs, ids, vals))
    mk = lambda dev: WideDeep(F, emb_dim=16, hidden=(64, 32), lr=0.3, dense_opt="adam", dense_lr=0.01,
                              world=World(device=torch.device(dev)), seed=4, device=dev)
    cpu, gpu = mk("cpu"), mk("cuda")
    for i, bt in enumerate(batches):
        lc = float(cpu.train_step(bt))
        lg = float(gpu.train_step(tuple(t.cuda() for t in bt)))
        assert abs(lc - lg) <= 1e-5 * max(1.0, abs(lc)), (i, lc, lg)
    for a, b in zip(cpu.dense_params, gpu.dense_params):
        assert torch.allclose(a, b.cpu(), atol=2e-5, rtol=1e-4)
    assert torch.allclose(cpu.emb.local, gpu.emb.local.cpu(), atol=2e-5)
    assert torch.allclose(cpu.wide.local, gpu.wide.local.cpu(), atol=2e-5)


def test_sparse_lr_fused_step_matches_general(monkeypatch):
    """One worker: the two-kernel step (csrc/kernels/sparse_lr.hip: no dedup,
    atomic scatter-SGD) trains like the general sharded path (radix-sort dedup,
    bag backward, owner-side apply) over 12 Zipf batches with hot ids."""
    import numpy as np

    from distributed_tensorflow_example_amd.models.sparse_lr import SparseLRTrainer
    from distributed_tensorflow_example_amd.parallel import world as W

    w = W.get_world() if W._WORLD is not None else W.init()
    rng = np.random.default_rng(4)
    B, F = 500, 1_000_000
    batches = []
    for _ in range(6):
        k = rng.integers(20, 61, B)
        offs = np.zeros(B + 1, np.int64)
        np.cumsum(k, out=offs[1:])
        ids = torch.from_numpy(((rng.zipf(1.1, int(offs[-1])) - 1) % F).astype(np.int64)).cuda()
        batches.append(((torch.rand(B, 1, device="cuda") < 0.3).float(), torch.from_numpy(offs).cuda(), ids,
                        torch.rand(int(offs[-1]), device="cuda")))
    monkeypatch.setenv("DTF_SLR_FUSED", "0")
    general = SparseLRTrainer(F, 1.0, w, seed=3)
    assert not general._fused_ok()
    monkeypatch.setenv("DTF_SLR_FUSED", "1")
    fused = SparseLRTrainer(F, 1.0, w, seed=3)
    assert fused._fused_ok()
    for i in range(12):
        lg = general.train_step(batches[i % 6])
        lf = fused.train_step(batches[i % 6])
        assert abs(float(lg) - float(lf)) < 1e-5, i
    assert fused.global_step == general.global_step == 12
    assert torch.allclose(general.W.local, fused.W.local, atol=1e-5)
    assert torch.allclose(general.b, fused.b, atol=1e-6)


@pytest.mark.gpu
def test_sparse_lr_fused_host_batches_match_device_batches():
    """Host (numpy / CPU tensor) batches take SparseLRPlan.run_csr -- one pinned
    pack + staging kernel -- and train exactly like the same batches on the GPU."""
    import numpy as np

    from distributed_tensorflow_example_amd.models.sparse_lr import SparseLRTrainer
    from distributed_tensorflow_example_amd.parallel import world as W

    w = W.get_world() if W._WORLD is not None else W.init()
    rng = np.random.default_rng(5)
    B, F = 300, 200_000
    host = []
    for _ in range(5):
        k = rng.integers(0, 50, B)
        offs = np.zeros(B + 1, np.int64)
        np.cumsum(k, out=offs[1:])
        ids = ((rng.zipf(1.2, int(offs[-1])) - 1) % F).astype(np.int64)
        host.append(((rng.random((B, 1)) < 0.4).astype(np.float32), offs, ids,
                     rng.random(int(offs[-1])).astype(np.float32)))
    dev = [tuple(torch.from_numpy(a).cuda() for a in b) for b in host]
    a = SparseLRTrainer(F, 0.5, w, seed=7)
    c = SparseLRTrainer(F, 0.5, w, seed=7)
    assert a._fused_ok()
    for i in range(10):
        hb = host[i % 5] if i % 2 == 0 else tuple(torch.from_numpy(x) for x in host[i % 5])
        la = float(a.train_step(hb))
        lc = float(c.train_step(dev[i % 5]))
        assert abs(la - lc) < 1e-6, i
    assert a._plan.timing()["runs"] == 10
    assert torch.equal(a.W.local, c.W.local) or torch.allclose(a.W.local, c.W.local, atol=1e-6)
    assert torch.allclose(a.b, c.b, atol=1e-7)
