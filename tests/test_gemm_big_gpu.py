"""Large-tile LDS-DMA MFMA GEMM (csrc/kernels/gemm_big.hip) vs a PyTorch fp32
reference of the same product, for every operand layout a linear layer uses
(forward x W^T, input gradient dY W, weight gradient dY^T X), bf16 and fp32
outputs, the bias / activation / beta epilogue, split-K and ragged M / N."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(A, tA, B, tB, bias=None, act=0, alpha=1.0, beta=0.0, C0=None):
    a = A.float().t() if tA else A.float()
    b = B.float().t() if tB else B.float()
    z = alpha * (a @ b)
    if bias is not None:
        z = z + bias
    if beta != 0.0:
        z = z + beta * C0.float()
    return {0: z, 1: torch.relu(z), 2: torch.sigmoid(z), 3: torch.tanh(z),
            4: torch.nn.functional.gelu(z)}[act]


def _operands(M, N, K, tA, tB, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    A = torch.randn(*((K, M) if tA else (M, K)), device="cuda", generator=g).bfloat16()
    B = torch.randn(*((N, K) if tB else (K, N)), device="cuda", generator=g).bfloat16()
    return A, B


def _rel(x, y):
    return float((x.float() - y).norm() / y.norm().clamp_min(1e-12))


@pytest.mark.parametrize("variant", [4, 8, 9])
@pytest.mark.parametrize("tA,tB", [(False, True), (False, False), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(512, 512, 256), (1000, 776, 192), (4096, 768, 768), (136, 264, 64),
                                   (1000, 776, 384), (136, 264, 128)])
def test_layouts_fp32_out(native, tA, tB, M, N, K, variant):
    if variant >= 8 and K % 128:
        pytest.skip("8-phase schedule: K % 128 == 0")
    A, B = _operands(M, N, K, tA, tB, M + N + K)
    C = torch.full((M, N), float("nan"), device="cuda")
    assert native.gemm_big(A, tA, B, tB, C, split_k=1, variant=variant)
    ref = _ref(A, tA, B, tB)
    # bf16 products are exact in fp32; only the summation order differs
    assert _rel(C, ref) < 1e-5, _rel(C, ref)


@pytest.mark.parametrize("variant", [8, 9])
@pytest.mark.parametrize("obf", [True, False])
@pytest.mark.parametrize("act", [0, 1, 2, 4])
def test_out_bias_act(native, act, obf, variant):
    M, N, K = 2048, 1024, 512
    A, B = _operands(M, N, K, False, True, act)
    bias = torch.randn(N, device="cuda")
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16 if obf else torch.float32)
    assert native.gemm_big(A, False, B, True, C, bias=bias, act=act, alpha=0.5, variant=variant)
    ref = _ref(A, False, B, True, bias, act, 0.5)
    assert _rel(C, ref) < (1e-2 if obf else 1e-5)


@pytest.mark.parametrize("variant,K", [(0, 320), (8, 384), (9, 384)])
@pytest.mark.parametrize("obf", [False, True])
def test_beta_accumulate(native, obf, variant, K):
    M, N = 768, 1280
    A, B = _operands(M, N, K, False, False, 7)
    dt = torch.bfloat16 if obf else torch.float32
    C0 = torch.randn(M, N, device="cuda").to(dt)
    C = C0.clone()
    assert native.gemm_big(A, False, B, False, C, beta=1.0, variant=variant)
    ref = _ref(A, False, B, False, beta=1.0, C0=C0)
    assert _rel(C, ref) < (1e-2 if obf else 1e-5)


@pytest.mark.parametrize("variant", [4, 8])
@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_split_k_weight_gradient(native, beta, variant):
    # dW[out, in] = dY^T X with T = 8192 tokens: few output tiles, long K
    T, O, I = 8192, 768, 768
    A, B = _operands(O, I, T, True, False, 11)
    C0 = torch.randn(O, I, device="cuda")
    C = C0.clone()
    assert native.gemm_big(A, True, B, False, C, beta=beta, split_k=0, variant=variant)
    ref = _ref(A, True, B, False, beta=beta, C0=C0)
    assert _rel(C, ref) < 1e-5


def test_contract_rejects_and_launches_nothing(native):
    A = torch.randn(256, 100, device="cuda").bfloat16()   # K % 64 != 0
    B = torch.randn(256, 100, device="cuda").bfloat16()
    C = torch.zeros(256, 256, device="cuda")
    assert not native.gemm_big(A, False, B, True, C)
    assert int(C.count_nonzero()) == 0


def test_linear_layer_products_match_torch(native):
    from distributed_tensorflow_example_amd.ops import big_gemm
    torch.manual_seed(0)
    x = torch.randn(4096, 768, device="cuda").bfloat16()
    w = (torch.randn(3072, 768, device="cuda") * 0.02).bfloat16()
    gy = torch.randn(4096, 3072, device="cuda").bfloat16()
    y = big_gemm.linear_fwd(x, w)
    assert _rel(y, x.float() @ w.float().t()) < 1e-2
    gx = big_gemm.linear_dx(gy, w)
    assert _rel(gx, gy.float() @ w.float()) < 1e-2
    dw = torch.zeros(3072, 768, device="cuda")
    big_gemm.linear_dw(gy, x, into=dw)
    assert _rel(dw, gy.float().t() @ x.float()) < 1e-5


@pytest.mark.parametrize("variant", [8, 9])
@pytest.mark.parametrize("tA,tB", [(False, True), (False, False), (True, False)])
@pytest.mark.parametrize("M,N,K", [(4096, 3072, 768), (16384, 768, 3072), (2304, 768, 4096)])
def test_8phase_race_screen(native, tA, tB, M, N, K, variant):
    """The 8-phase schedule's LDS hand-offs are placed by vmcnt / barrier count:
    a read placed one phase early passes reference checks whenever the DMA
    lands first, so every run of one shape must be bitwise identical (fixed
    summation order) and match the reference."""
    A, B = _operands(M, N, K, tA, tB, 5)
    C = torch.empty(M, N, device="cuda")
    assert native.gemm_big(A, tA, B, tB, C, split_k=1, variant=variant)
    first = C.clone()
    assert _rel(first, _ref(A, tA, B, tB)) < 1e-5
    for _ in range(12):
        C.fill_(float("nan"))
        native.gemm_big(A, tA, B, tB, C, split_k=1, variant=variant)
        assert torch.equal(C, first)
