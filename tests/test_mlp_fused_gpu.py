"""Fused MLP step kernels (csrc/kernels/mlp_step.hip) vs a PyTorch fp32 reference."""
import numpy as np
import pytest
import torch

from distributed_tensorflow_example_amd.data.mnist import PinnedEpoch, synthetic_mnist
from distributed_tensorflow_example_amd.models import mlp

pytestmark = pytest.mark.gpu


def _bf16(t):
    return t.to(torch.bfloat16).float()


def _ref(flat, x_u8, labels, act="sigmoid"):
    # reference with the same bf16 rounding of GEMM operands as the kernel
    x = _bf16(x_u8.float() / 255.0)
    f = flat.clone()
    f[: mlp.OFF_B1] = _bf16(f[: mlp.OFF_B1])
    return mlp.reference_loss_and_grad(f, x, labels, act)


@pytest.mark.parametrize("B", [100, 16, 37, 256, 1000])
@pytest.mark.parametrize("act", ["sigmoid", "relu"])
def test_fused_step_matches_reference(native, B, act):
    torch.manual_seed(0)
    imgs, labels = synthetic_mnist(B, seed=3)
    dev = torch.device("cuda")
    tr = mlp.FusedMLPTrainer(batch_size=B, lr=0.1, act=act, device=dev)
    p0 = tr.get_params().clone()
    x = torch.from_numpy(imgs).to(dev)
    y = torch.from_numpy(labels).to(dev)
    tr.step_tensors(x, y)
    torch.cuda.synchronize()
    loss, acc, g = _ref(p0, torch.from_numpy(imgs), torch.from_numpy(labels), act)
    m = tr.read_metrics(0, 1)[0]
    assert abs(m[0] - loss.item()) < 2e-2 * max(1.0, abs(loss.item())), (m, loss)
    assert abs(m[1] - acc.item()) < 0.05
    p1 = tr.get_params()
    g_k = (p0 - p1) / 0.1
    # bf16 GEMM operands: compare in relative Frobenius norm plus a loose max-abs bound
    rel = ((g_k - g).norm() / g.norm()).item()
    err = (g_k - g).abs().max().item()
    scale = g.abs().max().item()
    assert rel < 2e-2, rel
    assert err < 5e-2 * scale + 1e-4, (err, scale)
    assert tr.global_step == 1


def test_grad_mode_and_apply(native):
    B = 100
    imgs, labels = synthetic_mnist(B, seed=5)
    dev = torch.device("cuda")
    tr = mlp.FusedMLPTrainer(batch_size=B, lr=0.05, device=dev)
    p0 = tr.get_params().clone()
    x = torch.from_numpy(imgs).to(dev)
    y = torch.from_numpy(labels).to(dev)
    grads = torch.zeros(mlp.NPARAM, dtype=torch.float32, device=dev)
    C = native
    C.mlp_l1_fwd(x, 0, 0, B, tr.W1T, tr.z2p)
    C.mlp_head_bwd(tr.z2p, y, 0, B, tr.W2T, tr.W2N, tr.params, tr.dz2T, tr.partials, 1.0 / B, 0, False, tr.gstep)
    C.mlp_wgrad(x, 0, 0, tr.dz2T, B, tr.partials, tr.params, tr.W1T, tr.W2T, tr.W2N, grads, 1,
                tr.lr, tr.metrics, tr.gstep)
    torch.cuda.synchronize()
    _, _, g = _ref(p0, torch.from_numpy(imgs), torch.from_numpy(labels))
    assert (grads.cpu() - g).abs().max().item() < 2e-2 * g.abs().max().item() + 1e-4
    # params untouched in grad mode
    assert torch.equal(tr.get_params(), p0)
    C.mlp_apply_flat(tr.params, grads, tr.lr, 0.5, tr.W1T, tr.W2T, tr.W2N)
    torch.cuda.synchronize()
    ref = p0 - 0.05 * 0.5 * grads.cpu()
    assert torch.allclose(tr.get_params(), ref, atol=1e-6)
    # bf16 shadow consistent with master
    W1T = tr.W1T.view(112, 800)[:100, :784].float().cpu()
    assert torch.allclose(W1T.t(), _bf16(ref[:78400].view(784, 100)))


def test_runner_graph_equals_eager(native):
    B = 100
    imgs, labels = synthetic_mnist(3000, seed=11)
    ep = PinnedEpoch(imgs, labels, B)
    dev = torch.device("cuda")
    res = []
    for use_graph in (False, True):
        tr = mlp.FusedMLPTrainer(batch_size=B, lr=0.01, device=dev)
        r = mlp.MLPStepRunner(tr, ep, steps_per_graph=7, use_graph=use_graph)
        r.run(45)
        torch.cuda.synchronize()
        res.append((tr.get_params(), tr.read_metrics(0, 45)))
        assert tr.global_step == 45
    assert torch.equal(res[0][0], res[1][0])
    assert np.array_equal(res[0][1], res[1][1])


def test_training_converges(native):
    B = 100
    imgs, labels = synthetic_mnist(20000, seed=21)
    ep = PinnedEpoch(imgs, labels, B)
    tr = mlp.FusedMLPTrainer(batch_size=B, lr=0.05, device=torch.device("cuda"))
    r = mlp.MLPStepRunner(tr, ep, steps_per_graph=50)
    r.run(1000)
    torch.cuda.synchronize()
    m = tr.read_metrics(0, 1000)
    assert m[-50:, 0].mean() < m[:50, 0].mean() * 0.5
    assert m[-50:, 1].mean() > 0.8


@pytest.mark.parametrize("kind", [torch.float32, torch.bfloat16])
def test_float_inputs(native, kind):
    B = 64
    imgs, labels = synthetic_mnist(B, seed=9)
    dev = torch.device("cuda")
    tr = mlp.FusedMLPTrainer(batch_size=B, lr=0.1, device=dev)
    p0 = tr.get_params().clone()
    x = (torch.from_numpy(imgs).float() / 255.0).to(kind).to(dev)
    tr.step_tensors(x, torch.from_numpy(labels).to(dev))
    torch.cuda.synchronize()
    _, _, g = _ref(p0, torch.from_numpy(imgs), torch.from_numpy(labels))
    g_k = (p0 - tr.get_params()) / 0.1
    assert ((g_k - g).norm() / g.norm()).item() < 2e-2


def test_grad_mode_with_rccl_comm_in_graph(native):
    """GRAD mode (wgrad -> RCCL all-reduce -> flat SGD) on a 1-rank RCCL
    communicator, eager and hipGraph-captured: the multi-GPU code path."""
    from distributed_tensorflow_example_amd.parallel.world import World

    dev = torch.device("cuda")
    comm = native.RcclComm(native.rccl_unique_id(), 1, 0)
    w = World(rank=0, world_size=1, device=dev, backend="rccl", comm=comm)
    B = 100
    imgs, labels = synthetic_mnist(2000, seed=13)
    ep = PinnedEpoch(imgs, labels, B)
    res = []
    for grad_dtype in (torch.float32, torch.bfloat16):
        for use_graph in (False, True):
            tr = mlp.FusedMLPTrainer(batch_size=B, lr=0.01, device=dev, world=w,
                                     grad_dtype=grad_dtype)
            tr.world_size = 2  # force GRAD mode: all-reduce(sum) over 1 rank, scale 1/2
            tr.grads = torch.zeros(mlp.NPARAM, dtype=grad_dtype, device=dev)
            r = mlp.MLPStepRunner(tr, ep, steps_per_graph=5, use_graph=use_graph)
            r.run(10)
            torch.cuda.synchronize()
            res.append(tr.get_params())
            assert tr.global_step == 10
    # eager == graph for each grad dtype
    assert torch.equal(res[0], res[1])
    assert torch.equal(res[2], res[3])
    # fp32-grad DP path with lr scaled by 1/world == fused path at lr/2
    tr = mlp.FusedMLPTrainer(batch_size=B, lr=0.005, device=dev)
    r = mlp.MLPStepRunner(tr, ep, steps_per_graph=5, use_graph=False)
    r.run(10)
    torch.cuda.synchronize()
    assert torch.allclose(tr.get_params(), res[0], atol=1e-5)
