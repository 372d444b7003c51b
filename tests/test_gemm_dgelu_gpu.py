"""gemm_big's GELU-backward epilogue (csrc/kernels/gemm_big.hip gemm_8ph<DG>,
binding gemm_dgelu) and BERT's fused FFN-down op against fp32 PyTorch
references: dU = (dY W) * gelu'(u + b) and db = colsum(dU)."""
import pytest
import torch

from distributed_tensorflow_example_amd.ops.transformer import gelu_ref

pytestmark = pytest.mark.gpu


def _gelu_grad_ref(z):
    z = z.detach().requires_grad_(True)
    gelu_ref(z).sum().backward()
    return z.grad


@pytest.mark.parametrize("M,N,K", [(512, 512, 256), (2048, 3072, 768), (768, 256, 128)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_gemm_dgelu_matches_fp32(native, M, N, K, accumulate):
    torch.manual_seed(0)
    bf = torch.bfloat16
    dy = torch.randn(M, K, device="cuda").to(bf)
    w = (torch.randn(K, N, device="cuda") * K ** -0.5).to(bf)
    u = torch.randn(M, N, device="cuda").to(bf)
    b = torch.randn(N, device="cuda") * 0.1
    du = torch.empty(M, N, device="cuda", dtype=bf)
    colpart = torch.empty((M // 128) * N, device="cuda")
    db0 = torch.randn(N, device="cuda")
    db = db0.clone()
    assert native.gemm_dgelu(dy, False, w, False, du, u, b, colpart, db, accumulate=accumulate)
    dh = dy.float() @ w.float()
    ref = dh * _gelu_grad_ref(u.float() + b)
    torch.testing.assert_close(du.float(), ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())
    dbr = ref.sum(0) + (db0 if accumulate else 0)
    torch.testing.assert_close(db, dbr, rtol=1e-3, atol=1e-3 * ref.abs().sum(0).max().item())


def test_gemm_dgelu_refuses_off_contract(native):
    bf = torch.bfloat16
    dy = torch.randn(300, 256, device="cuda").to(bf)
    w = torch.randn(256, 512, device="cuda").to(bf)
    u = torch.randn(300, 512, device="cuda").to(bf)
    du = torch.empty_like(u)
    b, db = torch.zeros(512, device="cuda"), torch.zeros(512, device="cuda")
    assert not native.gemm_dgelu(dy, False, w, False, du, u, b, torch.empty(3 * 512, device="cuda"), db)


@pytest.mark.parametrize("M,N,K", [(512, 512, 256), (2048, 3072, 768)])
def test_gemm_gelu_aux_matches_fp32(native, M, N, K):
    torch.manual_seed(2)
    bf = torch.bfloat16
    x = torch.randn(M, K, device="cuda").to(bf)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(bf)
    b = torch.randn(N, device="cuda") * 0.1
    u, h = torch.empty(M, N, device="cuda", dtype=bf), torch.empty(M, N, device="cuda", dtype=bf)
    assert native.gemm_gelu_aux(x, False, w, True, h, u, b)
    ur = x.float() @ w.float().t() + b
    torch.testing.assert_close(u.float(), ur, rtol=1e-2, atol=1e-2 * ur.abs().max().item())
    hr = gelu_ref(ur)
    torch.testing.assert_close(h.float(), hr, rtol=1e-2, atol=1e-2 * hr.abs().max().item())


def test_gemm_dgelu_without_bias(native):
    torch.manual_seed(3)
    bf = torch.bfloat16
    dy = torch.randn(512, 256, device="cuda").to(bf)
    w = (torch.randn(256, 512, device="cuda") * 0.0625).to(bf)
    u = torch.randn(512, 512, device="cuda").to(bf)
    du, db = torch.empty_like(u), torch.empty(512, device="cuda")
    assert native.gemm_dgelu(dy, False, w, False, du, u, None, torch.empty(4 * 512, device="cuda"), db)
    ref = (dy.float() @ w.float()) * _gelu_grad_ref(u.float())
    torch.testing.assert_close(du.float(), ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())
    torch.testing.assert_close(db, ref.sum(0), rtol=1e-3, atol=1e-3 * ref.abs().sum(0).max().item())


@pytest.mark.parametrize("policy", ["always", "never"])
def test_bert_fused_ffn_matches_fp32(native, monkeypatch, policy):
    """models/bert.py _FFN (fused GELU epilogues under 'always', the separate
    passes under 'never') vs gelu(x W1^T + b1) W2^T in fp32 autograd: the
    output and the x, W1, b1, W2 gradients."""
    from distributed_tensorflow_example_amd.models import bert
    from distributed_tensorflow_example_amd.ops import big_gemm

    monkeypatch.setattr(big_gemm, "_POLICY", policy)
    torch.manual_seed(1)
    M, D, F_ = 1024, 256, 512
    x = torch.randn(M, D, device="cuda").to(torch.bfloat16).requires_grad_(True)
    w1 = (torch.randn(F_, D, device="cuda") * D ** -0.5).requires_grad_(True)
    b1 = (torch.randn(F_, device="cuda") * 0.1).requires_grad_(True)
    w2 = (torch.randn(D, F_, device="cuda") * F_ ** -0.5).requires_grad_(True)
    for w in (w1, w2):
        w._shadow = w.detach().to(torch.bfloat16)
    y = bert._ffn(x, w1, b1, w2)
    g = torch.randn(M, D, device="cuda").to(torch.bfloat16)
    y.backward(g)
    xr = x.detach().float().requires_grad_(True)
    w1r = w1._shadow.float().requires_grad_(True)
    b1r = b1.detach().clone().requires_grad_(True)
    w2r = w2._shadow.float().requires_grad_(True)
    yr = gelu_ref(xr @ w1r.t() + b1r) @ w2r.t()
    yr.backward(g.float())
    for got, ref in ((y.float(), yr), (x.grad.float(), xr.grad), (w1.grad, w1r.grad), (b1.grad, b1r.grad),
                     (w2.grad, w2r.grad)):
        torch.testing.assert_close(got, ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
