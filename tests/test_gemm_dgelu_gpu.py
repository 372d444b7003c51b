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


@pytest.mark.parametrize("policy", ["always", "never"])
def test_bert_fused_ffn_down_matches_unfused(native, monkeypatch, policy):
    """_GeluShadowLinear (fused epilogue or fallback) vs bias_gelu + linear in
    fp32 autograd: input, bias and weight gradients."""
    from distributed_tensorflow_example_amd.models import bert
    from distributed_tensorflow_example_amd.ops import big_gemm

    monkeypatch.setattr(big_gemm, "_POLICY", policy)
    torch.manual_seed(1)
    M, H, O = 1024, 512, 256
    u = torch.randn(M, H, device="cuda").to(torch.bfloat16).requires_grad_(True)
    b = (torch.randn(H, device="cuda") * 0.1).requires_grad_(True)
    w = (torch.randn(O, H, device="cuda") * H ** -0.5).requires_grad_(True)
    w._shadow = w.detach().to(torch.bfloat16)
    y = bert._gelu_mm(u, b, w)
    g = torch.randn(M, O, device="cuda").to(torch.bfloat16)
    y.backward(g)
    ur = u.detach().float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    wr = w._shadow.float().requires_grad_(True)
    yr = gelu_ref(ur + br) @ wr.t()
    yr.backward(g.float())
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2 * yr.abs().max().item())
    torch.testing.assert_close(u.grad.float(), ur.grad, rtol=2e-2, atol=2e-2 * ur.grad.abs().max().item())
    torch.testing.assert_close(b.grad, br.grad, rtol=2e-2, atol=2e-2 * br.grad.abs().max().item())
    torch.testing.assert_close(w.grad, wr.grad, rtol=2e-2, atol=2e-2 * wr.grad.abs().max().item())
