"""ResNet-side kernels against plain PyTorch fp32 references: the NHWC bf16
max pool (csrc/kernels/pool.hip) and the 1x1 convolution weight gradient on
the in-tree GEMM (ops/conv.py)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape,k,s,p", [((4, 64, 112, 112), 3, 2, 1), ((2, 16, 9, 11), 3, 2, 1),
                                         ((2, 8, 10, 10), 2, 2, 0), ((1, 24, 7, 7), 3, 1, 1),
                                         ((2, 8, 9, 12), 3, 2, 0)])
def test_maxpool_nhwc_matches_fp32(native, shape, k, s, p):
    from distributed_tensorflow_example_amd.ops.pool import max_pool2d

    torch.manual_seed(0)
    x = torch.randn(shape, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    y = max_pool2d(x, k, s, p)
    xr = x.detach().float().requires_grad_(True)
    yr = F.max_pool2d(xr, k, s, p)
    assert y.shape == yr.shape
    assert torch.equal(y.float(), yr)                       # a max of bf16 values is exact
    g = torch.randn_like(yr)
    y.backward(g.to(torch.bfloat16))
    yr.backward(g.to(torch.bfloat16).float())
    # random inputs: no ties, so every gradient lands on the same input as torch's
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=1e-2, atol=1e-2)


def test_maxpool_ties_take_first_and_nan_propagates(native):
    from distributed_tensorflow_example_amd.ops.pool import max_pool2d

    x = torch.zeros(1, 8, 4, 4, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x[0, 0, 1, 1] = float("nan")
    x.requires_grad_(True)
    y = max_pool2d(x, 2, 2, 0)
    assert torch.isnan(y[0, 0, 0, 0]) and torch.all(y[0, 1:] == 0)
    y.backward(torch.ones_like(y))
    # all-zero windows: the first position (0, 0) of each window gets the gradient
    assert x.grad[0, 1, 0, 0] == 1 and x.grad[0, 1, 0, 1] == 0 and x.grad[0, 1, 1, 0] == 0


def test_maxpool_3x3_stride2_ties_match_torch(native):
    """The specialized 3x3 / stride-2 kernels on tie-heavy input (all zeros with a
    NaN): torch's first-maximum rule, forward values and the gradient routing."""
    from distributed_tensorflow_example_amd.ops.pool import max_pool2d

    x = torch.zeros(2, 16, 11, 13, device="cuda", dtype=torch.bfloat16)
    x[1, 3, 4, 5] = float("nan")
    x = x.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = max_pool2d(x, 3, 2, 1)
    xr = x.detach().float().requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    torch.testing.assert_close(y.float(), yr, equal_nan=True, rtol=0, atol=0)
    g = torch.arange(yr.numel(), device="cuda", dtype=torch.float32).reshape(yr.shape).remainder(7).bfloat16()
    y.backward(g.contiguous(memory_format=torch.channels_last))
    yr.backward(g.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=0, atol=0)


@pytest.mark.parametrize("engines", [("hipblaslt", "hipblaslt", "gemm_big"), ("gemm_big", "gemm_big", "gemm_big"),
                                     ("miopen", "miopen", "miopen"), ("miopen", "hipblaslt", "miopen")])
@pytest.mark.parametrize("n,cin,cout,hw", [(8, 64, 256, 28), (4, 256, 64, 14), (16, 512, 128, 7)])
def test_conv1x1_engines_match_fp32(native, n, cin, cout, hw, engines):
    """Every engine choice of the 1x1 convolution's three products (ops/conv.py)
    against an fp32 einsum reference."""
    from distributed_tensorflow_example_amd.ops import conv

    torch.manual_seed(1)
    m = conv.ShadowConv2d(cin, cout, 1, bias=False).cuda().to(memory_format=torch.channels_last)
    conv.attach_shadows(m)
    x = torch.randn(n, cin, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    key = (tuple(x.shape), cout)
    for role, eng in zip(("fwd", "dx", "dw"), engines):
        conv._choice[(role,) + key] = eng
    try:
        x.requires_grad_(True)
        y = m(x)
        assert y.is_contiguous(memory_format=torch.channels_last)
        g = torch.randn_like(y.float()).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y.backward(g)
    finally:
        for role in ("fwd", "dx", "dw"):
            conv._choice.pop((role,) + key, None)
    xr = x.detach().float()
    wr = m.weight.detach().to(torch.bfloat16).float().view(cout, cin)
    gr = g.float()
    y_ref = torch.einsum("nihw,oi->nohw", xr, wr)
    dw_ref = torch.einsum("nohw,nihw->oi", gr, xr).view_as(m.weight)
    dx_ref = torch.einsum("nohw,oi->nihw", gr, wr)
    torch.testing.assert_close(y.float(), y_ref, rtol=2e-2, atol=2e-2 * y_ref.abs().max().item())
    torch.testing.assert_close(m.weight.grad, dw_ref, rtol=2e-3, atol=2e-3 * dw_ref.abs().max().item())
    torch.testing.assert_close(x.grad.float(), dx_ref, rtol=2e-2, atol=2e-2 * dx_ref.abs().max().item())


@pytest.mark.parametrize("dx_engine", ["hipblaslt", "gemm_big", "miopen"])
def test_bottleneck_residual_grad_fold(native, dx_engine):
    """An identity bottleneck's residual gradient accumulated by conv1's dx GEMM
    (beta = 1, models/resnet.py) equals autograd's two-branch sum."""
    from distributed_tensorflow_example_amd.models.resnet import Bottleneck
    from distributed_tensorflow_example_amd.ops import conv

    torch.manual_seed(3)
    blk = Bottleneck(256, 64).cuda().to(memory_format=torch.channels_last).train()
    conv.attach_shadows(blk)
    x0 = torch.randn(8, 256, 14, 14, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = torch.randn(8, 256, 14, 14, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    key = ("dx", tuple(x0.shape), 64)
    conv._choice[key] = dx_engine
    grads = []
    try:
        for fold in (True, False):
            blk.fold_residual_grad = fold
            blk.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            blk(x).backward(g)
            grads.append((x.grad.float(), blk.conv1.weight.grad.clone()))
    finally:
        conv._choice.pop(key, None)
        blk.fold_residual_grad = True
    (a, wa), (b, wb) = grads
    # one bf16 rounding of (dy W + dres) vs two (dy W, then the add)
    torch.testing.assert_close(a, b, rtol=1e-2, atol=1e-2 * b.abs().max().item())
    torch.testing.assert_close(wa, wb)


def test_bottleneck_fold_off_without_shadows(native):
    """Without bf16 shadows conv1 runs as plain nn.Conv2d and cannot take the
    residual gradient, so no slot is created: gradients match the unfolded block."""
    from distributed_tensorflow_example_amd.models.resnet import Bottleneck

    torch.manual_seed(4)
    blk = Bottleneck(64, 16).cuda().to(memory_format=torch.channels_last).train()
    x = torch.randn(2, 64, 8, 8, device="cuda").contiguous(memory_format=torch.channels_last)
    assert not blk._fold_ok(x)
    xr = x.clone().requires_grad_(True)
    blk(xr).float().sum().backward()
    grads = xr.grad.clone()
    blk.fold_residual_grad = False
    xr2 = x.clone().requires_grad_(True)
    blk.zero_grad(set_to_none=True)
    blk(xr2).float().sum().backward()
    blk.fold_residual_grad = True
    assert torch.equal(grads, xr2.grad)


@pytest.mark.parametrize("stride,cin,hw", [(2, 256, 28), (1, 64, 28), (2, 512, 15)])
def test_downsample_block_input_grad_share(native, stride, cin, hw):
    """A downsampling bottleneck's conv1 / projection input gradients folded into
    one tensor (ops/conv.py XGradShare: GEMM beta = 1, or the stride-2
    projection's strided pixels via strided_add) equal autograd's sum."""
    from distributed_tensorflow_example_amd.models.resnet import Bottleneck
    from distributed_tensorflow_example_amd.ops import conv

    torch.manual_seed(5)
    blk = Bottleneck(cin, 64, stride=stride, down=True).cuda().to(memory_format=torch.channels_last).train()
    conv.attach_shadows(blk)
    x0 = torch.randn(4, cin, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    grads = []
    for fold in (True, False):
        blk.share_input_grad = fold
        blk.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        assert blk._share_ok(x) == fold
        y = blk(x)
        y.backward(torch.ones_like(y) * 0.01)
        grads.append((x.grad.float(), blk.conv1.weight.grad.clone(), blk.down_conv.weight.grad.clone()))
    blk.share_input_grad = True
    (a, w1a, wda), (b, w1b, wdb) = grads
    torch.testing.assert_close(a, b, rtol=1e-2, atol=1e-2 * b.abs().max().item())
    # weight gradients: same kernels, but MIOpen's split-K weight-gradient solvers
    # accumulate with atomics (bf16 results may differ by an ulp run to run)
    torch.testing.assert_close(w1a, w1b, rtol=1e-2, atol=1e-2 * w1b.abs().max().item())
    torch.testing.assert_close(wda, wdb, rtol=1e-2, atol=1e-2 * wdb.abs().max().item())


def test_strided_add_matches_torch(native):
    torch.manual_seed(6)
    full = torch.randn(2, 16, 9, 9, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    comp = torch.randn(2, 16, 5, 5, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ref = full.float().clone()
    ref[:, :, ::2, ::2] += comp.float()
    native.strided_add(full, comp, 2)
    torch.testing.assert_close(full.float(), ref.bfloat16().float())
