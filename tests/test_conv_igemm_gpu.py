"""In-tree 3x3 implicit-GEMM convolution (csrc/kernels/conv_igemm.hip) against
torch's fp32 conv2d of the same bf16 operands: forward at stride 1 / 2 (odd
spatial sizes, partial last tile, both channel tilings), the BatchNorm
statistics partials of its output, and the stride-1 input gradient through
the flipped filter; the ShadowConv2d autograd path on it."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def _close(got, ref, tol=1e-2):
    err = (got.float() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= tol * scale + 1e-3, (err, scale)


@pytest.mark.parametrize("N,C,H,W,K,s", [(2, 64, 14, 14, 64, 1), (3, 128, 9, 7, 192, 1), (2, 64, 15, 13, 128, 2),
                                         (1, 256, 7, 7, 256, 1), (4, 64, 8, 8, 64, 2)])
def test_conv3x3_forward_matches_fp32(N, C, H, W, K, s):
    from distributed_tensorflow_example_amd.ops import conv

    g = torch.Generator(device="cuda").manual_seed(N * 1000 + C + K + s)
    x = _cl(torch.randn(N, C, H, W, device="cuda", generator=g).bfloat16())
    w = _cl((torch.randn(K, C, 3, 3, device="cuda", generator=g) * (2.0 / (9 * C)) ** 0.5).bfloat16())
    assert conv.igemm_ok(x, w, (s, s), (1, 1), (1, 1), 1)
    P = conv.conv3x3_stat_rows(x, s)
    part = torch.full((2, P, K), float("nan"), device="cuda")
    y = conv.conv3x3(x, w, s, stats=part)
    ref = F.conv2d(x.float(), w.float(), None, s, 1)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    _close(y, ref)
    # BN statistics of the bf16 output, per channel
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, K)
    torch.testing.assert_close(part[0].sum(0), yf.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(part[1].sum(0), (yf * yf).sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("N,C,H,W,K", [(2, 64, 12, 10, 128), (2, 128, 7, 7, 64)])
def test_conv3x3_input_gradient_matches_fp32(N, C, H, W, K):
    from distributed_tensorflow_example_amd.ops import conv

    g = torch.Generator(device="cuda").manual_seed(7 + C + K)
    x = _cl(torch.randn(N, C, H, W, device="cuda", generator=g).bfloat16())
    w = _cl((torch.randn(K, C, 3, 3, device="cuda", generator=g) * 0.05).bfloat16())
    dy = _cl(torch.randn(N, K, H, W, device="cuda", generator=g).bfloat16())
    dx = conv.conv3x3_dx(dy, w, x.shape)
    xr = x.float().requires_grad_(True)
    F.conv2d(xr, w.float(), None, 1, 1).backward(dy.float())
    _close(dx, xr.grad)


def test_shadow_conv_on_igemm_trains_like_miopen(monkeypatch):
    """ShadowConv2d (3x3, stride 1) forced onto the in-tree kernel: output and
    both gradients match the MIOpen path of the same module."""
    from distributed_tensorflow_example_amd.ops import conv

    torch.manual_seed(0)
    res = {}
    for mode in ("always", "never"):
        monkeypatch.setattr(conv, "_IGEMM", mode)
        m = conv.ShadowConv2d(64, 64, 3, 1, 1, bias=False).cuda().to(memory_format=torch.channels_last)
        with torch.no_grad():
            m.weight.copy_(torch.linspace(-0.05, 0.05, m.weight.numel(), device="cuda").view_as(m.weight))
        conv.attach_shadows(m)
        x = _cl(torch.linspace(-1, 1, 2 * 64 * 10 * 10, device="cuda").view(2, 64, 10, 10).sin().bfloat16())
        x.requires_grad_(True)
        y = m(x)
        y.float().square().sum().backward()
        res[mode] = (y.float(), x.grad.float(), m.weight.grad.float())
    for a, b in zip(res["always"], res["never"]):
        _close(a, b, 2e-2)


@pytest.mark.parametrize("N,C,H,W,K,s,cl", [(2, 64, 12, 10, 64, 1, True), (2, 128, 9, 7, 192, 1, False),
                                            (3, 64, 15, 13, 128, 2, True), (2, 256, 7, 7, 128, 1, False)])
def test_conv3x3_weight_gradient_matches_fp32(N, C, H, W, K, s, cl):
    """Split-K weight gradient accumulated into an fp32 buffer (channels_last or
    contiguous) that already holds a gradient."""
    from distributed_tensorflow_example_amd.ops import conv

    g = torch.Generator(device="cuda").manual_seed(11 + C + K + s)
    x = _cl(torch.randn(N, C, H, W, device="cuda", generator=g).bfloat16())
    Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
    dy = _cl(torch.randn(N, K, Ho, Wo, device="cuda", generator=g).bfloat16())
    w = torch.zeros(K, C, 3, 3, device="cuda", requires_grad=True)
    F.conv2d(x.float(), w, None, s, 1).backward(dy.float())
    prior = torch.randn(K, C, 3, 3, device="cuda", generator=g)
    into = prior.clone().contiguous(memory_format=torch.channels_last if cl else torch.contiguous_format)
    conv.conv3x3_dw(dy, x, s, into=into)
    _close(into - prior, w.grad, 2e-3)


def test_conv_bn_statistics_handoff(monkeypatch):
    """3x3 conv on the in-tree kernel -> FusedBatchNorm2d(relu): the BN takes the
    statistics partials from the conv's epilogue (no statistics pass) and gives
    the same output, running stats and gradients as the plain path."""
    from distributed_tensorflow_example_amd.ops import conv
    from distributed_tensorflow_example_amd.ops.bn import FusedBatchNorm2d

    monkeypatch.setattr(conv, "_IGEMM", "always")
    res = {}
    for stats in (True, False):
        monkeypatch.setattr(conv, "_BN_STATS", stats)
        torch.manual_seed(3)
        m = conv.ShadowConv2d(64, 128, 3, 2, 1, bias=False).cuda().to(memory_format=torch.channels_last)
        bn = FusedBatchNorm2d(128).cuda()
        conv.attach_shadows(m)
        x = _cl(torch.randn(4, 64, 15, 15, device="cuda").bfloat16()).requires_grad_(True)
        y = m(x)
        assert hasattr(y, "_dtf_bn_part") == stats
        out = bn(y, relu=True)
        out.float().square().sum().backward()
        res[stats] = (out.float(), bn.running_mean.clone(), bn.running_var.clone(), x.grad.float(),
                      m.weight.grad.float(), bn.weight.grad.float())
    for a, b in zip(res[True], res[False]):
        _close(a, b, 1e-2)


def test_conv_bn_statistics_handoff_ignored_after_inplace_write(monkeypatch):
    """An in-place write to the conv output between the conv and the BN (y += r)
    bumps its version: the BN must not use the conv epilogue's statistics of the
    old values -- it recomputes them and matches the plain BN of the new y."""
    from distributed_tensorflow_example_amd.ops import conv
    from distributed_tensorflow_example_amd.ops.bn import FusedBatchNorm2d

    monkeypatch.setattr(conv, "_IGEMM", "always")
    monkeypatch.setattr(conv, "_BN_STATS", True)
    torch.manual_seed(5)
    m = conv.ShadowConv2d(64, 128, 3, 1, 1, bias=False).cuda().to(memory_format=torch.channels_last)
    conv.attach_shadows(m)
    x = _cl(torch.randn(4, 64, 12, 12, device="cuda").bfloat16())
    r = _cl(torch.randn(4, 128, 12, 12, device="cuda").bfloat16()) * 3 + 1
    with torch.no_grad():
        y = m(x)
        assert hasattr(y, "_dtf_bn_part")
        y += r
        out = FusedBatchNorm2d(128).cuda()(y, relu=True)
        yf = y.float()
        mu = yf.mean(dim=(0, 2, 3), keepdim=True)
        var = yf.var(dim=(0, 2, 3), unbiased=False, keepdim=True)
        ref = torch.relu((yf - mu) / torch.sqrt(var + 1e-5))
    _close(out.float(), ref, 2e-2)


@pytest.mark.parametrize("ks,two_consumers", [(3, False), (1, False), (3, True)])
def test_bn_backward_partials_from_conv_input_gradient(monkeypatch, ks, two_consumers):
    """FusedBatchNorm2d(relu) -> conv (3x3 or 1x1, in-tree implicit GEMM): the
    conv's input-gradient epilogue masks the gradient with the ReLU and writes
    the BN backward's partials, and the BN finalizes from them.  Output and all
    gradients match the unfused path; with a second consumer of the BN output
    (autograd sums into the gradient) the BN falls back to its own pass."""
    from distributed_tensorflow_example_amd.ops import bn as bn_mod
    from distributed_tensorflow_example_amd.ops import conv
    from distributed_tensorflow_example_amd.ops.bn import FusedBatchNorm2d

    monkeypatch.setattr(conv, "_IGEMM", "always")
    N, C, H, W, K = 4, 64, 16, 16, 128
    key = ((N, C, H, W), K)
    monkeypatch.setattr(conv, "_choice", {("fwd",) + key: "igemm", ("dx",) + key: "igemm", ("dw",) + key: "igemm"})
    taken = []
    orig = bn_mod.BwdSlot.take

    def spy(self, dy):
        r = orig(self, dy)
        taken.append(r is not None)
        return r
    monkeypatch.setattr(bn_mod.BwdSlot, "take", spy)
    res = {}
    for fused in (True, False):
        monkeypatch.setattr(bn_mod, "_BWD_EPI", fused)
        taken.clear()
        torch.manual_seed(5)
        bn = FusedBatchNorm2d(C).cuda()
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.3, 0.3)
        m = conv.ShadowConv2d(C, K, ks, 1, ks // 2, bias=False).cuda().to(memory_format=torch.channels_last)
        conv.attach_shadows(m)
        x = _cl(torch.randn(N, C, H, W, device="cuda").bfloat16()).requires_grad_(True)
        h = bn(x, relu=True)
        assert hasattr(h, "_dtf_bn_bwd") == fused
        y = m(h)
        loss = y.float().square().sum()
        if two_consumers:
            loss = loss + (h.float() * torch.linspace(-1, 1, W, device="cuda")).sum()
        loss.backward()
        if fused:
            assert taken == [not two_consumers], taken
        res[fused] = (y.float(), x.grad.float(), bn.weight.grad.float(), bn.bias.grad.float(), m.weight.grad.float())
    for a, b in zip(res[True], res[False]):
        _close(a, b, 1.5e-2)


def test_bottleneck_chain_bn_backward_epilogues(monkeypatch):
    """Three identity bottlenecks (models/resnet.py) with every conv on the
    implicit GEMM: bn1 / bn2 take their backward partials from conv2 / conv3's
    input-gradient epilogue, and each block's bn3 (residual + ReLU) from the
    next block's conv1, whose input gradient is added onto the folded residual
    gradient first.  Output, input gradient and every parameter gradient match
    the unfused path."""
    from distributed_tensorflow_example_amd.models.resnet import Bottleneck
    from distributed_tensorflow_example_amd.ops import bn as bn_mod
    from distributed_tensorflow_example_amd.ops import conv

    monkeypatch.setattr(conv, "_IGEMM", "always")
    N, H = 4, 16
    ch = {}
    for cin, cout in ((256, 64), (64, 256)):
        key = ((N, cin, H, H), cout)
        for role in ("fwd", "dx", "dw"):
            ch[(role,) + key] = "igemm"
    monkeypatch.setattr(conv, "_choice", ch)
    taken = []
    orig = bn_mod.BwdSlot.take

    def spy(self, dy):
        r = orig(self, dy)
        taken.append((self.res is not None, r is not None))
        return r
    monkeypatch.setattr(bn_mod.BwdSlot, "take", spy)
    res = {}
    for fused in (True, False):
        monkeypatch.setattr(bn_mod, "_BWD_EPI", fused)
        taken.clear()
        torch.manual_seed(9)
        net = torch.nn.Sequential(*[Bottleneck(256, 64) for _ in range(3)]).cuda().to(
            memory_format=torch.channels_last)
        for m in net.modules():
            if isinstance(m, bn_mod.FusedBatchNorm2d):
                with torch.no_grad():
                    m.weight.uniform_(0.5, 1.5)
                    m.bias.uniform_(-0.2, 0.2)
        conv.attach_shadows(net)
        x = _cl(torch.randn(N, 256, H, H, device="cuda").bfloat16()).requires_grad_(True)
        y = net(x)
        (y.float() * torch.linspace(-1, 1, H, device="cuda")).square().sum().backward()
        if fused:
            # 3 blocks x (bn1, bn2) plain + bn3 of blocks 0 and 1 through the next conv1
            assert sum(1 for r, t in taken if t and not r) == 6, taken
            assert sum(1 for r, t in taken if t and r) == 2, taken
        grads = [p.grad.float().clone() for p in net.parameters()]
        res[fused] = [y.float(), x.grad.float()] + grads
    for a, b in zip(res[True], res[False]):
        _close(a, b, 2e-2)


@pytest.mark.parametrize("M,K,N", [(2 * 256, 256, 512), (6272, 512, 2048), (3136 // 2, 256, 64), (200, 128, 136)])
def test_gemm_bn_stats_epilogue(M, K, N):
    """gemm_big's statistics epilogue (dtfk_gemm_bn_stats): y = x W^T in bf16 and
    the per-128-row column sums / sums of squares of the STORED y, interior and
    edge tiles (M % 256 != 0, N % 256 != 0), against fp32 sums of y itself."""
    from distributed_tensorflow_example_amd import _native

    C = _native.load()
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    P = int(C.gemm_bn_stat_rows(M))
    part = torch.full((2, P, N), float("nan"), device="cuda")
    assert C.gemm_bn_stats(x, False, w, True, y, part)
    ref = x.float() @ w.float().t()
    _close(y.float(), ref, 1e-2)
    yf = y.float()
    pad = torch.zeros(P * 128 - M, N, device="cuda")
    yb = torch.cat([yf, pad]).view(P, 128, N)
    torch.testing.assert_close(part[0], yb.sum(1), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(part[1], yb.square().sum(1), rtol=1e-4, atol=1e-3)


def test_conv1x1_bn_statistics_handoff(monkeypatch):
    """1x1 conv on gemm_big with the statistics epilogue -> FusedBatchNorm2d(relu):
    same output, running stats and gradients as the plain path (stats pass in the BN)."""
    from distributed_tensorflow_example_amd.ops import conv
    from distributed_tensorflow_example_amd.ops.bn import FusedBatchNorm2d

    res = {}
    for stats in (True, False):
        monkeypatch.setattr(conv, "_BN_STATS", stats)
        conv._choice.clear()
        torch.manual_seed(5)
        m = conv.ShadowConv2d(256, 128, 1, 1, 0, bias=False).cuda().to(memory_format=torch.channels_last)
        bn = FusedBatchNorm2d(128).cuda()
        conv.attach_shadows(m)
        x = _cl(torch.randn(4, 256, 16, 16, device="cuda").bfloat16()).requires_grad_(True)
        key = ("fwd", tuple(x.shape), 128)
        conv._choice[key] = "gemm_big"
        y = m(x)
        assert hasattr(y, "_dtf_bn_part") == stats
        out = bn(y, relu=True)
        out.float().square().sum().backward()
        res[stats] = (out.float(), bn.running_mean.clone(), bn.running_var.clone(), x.grad.float(),
                      m.weight.grad.float(), bn.weight.grad.float())
    conv._choice.clear()
    for a, b in zip(res[True], res[False]):
        _close(a, b, 1e-2)


def test_strided_1x1_conv_gathered_gemms_match_conv2d(monkeypatch):
    """A stride-2 1x1 ShadowConv2d (ResNet's projection) with its forward and
    weight gradient as GEMMs over the gathered strided pixels: output, input
    and weight gradients match nn.functional.conv2d in fp32."""
    from distributed_tensorflow_example_amd.ops import conv

    monkeypatch.setattr(conv, "_S2_GATHER", True)
    torch.manual_seed(9)
    m = conv.ShadowConv2d(128, 256, 1, 2, 0, bias=False).cuda().to(memory_format=torch.channels_last)
    conv.attach_shadows(m)
    x = _cl(torch.randn(4, 128, 16, 16, device="cuda").bfloat16()).requires_grad_(True)
    xs_shape = (4, 128, 8, 8)
    conv._choice.clear()
    conv._choice[("fwd", xs_shape, 256)] = "gemm_big"
    conv._choice[("dw", xs_shape, 256)] = "gemm_big"
    try:
        y = m(x)
        dy = _cl(torch.randn_like(y.float()).bfloat16())
        y.backward(dy)
    finally:
        conv._choice.clear()
    w = m.weight._shadow.float().detach().requires_grad_(True)
    xr = x.detach().float().requires_grad_(True)
    ref = F.conv2d(xr, w, None, 2)
    ref.backward(dy.float())
    _close(y, ref)
    _close(x.grad, xr.grad)
    _close(m.weight.grad, w.grad)


@pytest.mark.parametrize("H,W", [(16, 16), (15, 13)])
def test_strided_1x1_conv_on_implicit_gemm_matches_conv2d(monkeypatch, H, W):
    """DTF_CONV_S2_GATHER=0: the stride-2 1x1 projection runs its forward (+ the BN
    statistics hand-off) and weight gradient on the implicit GEMM's strided loads
    (no gathered copy); output and both gradients match fp32 conv2d."""
    from distributed_tensorflow_example_amd.ops import conv

    monkeypatch.setattr(conv, "_S2_GATHER", False)
    torch.manual_seed(13)
    m = conv.ShadowConv2d(128, 256, 1, 2, 0, bias=False).cuda().to(memory_format=torch.channels_last)
    conv.attach_shadows(m)
    x = _cl(torch.randn(4, 128, H, W, device="cuda").bfloat16()).requires_grad_(True)
    assert conv.igemm_ok(x, m.weight._shadow, (2, 2), (0, 0), (1, 1), 1)
    conv._choice.clear()
    key = (tuple(x.shape), 256, 2, 1)
    conv._choice[("fwd3",) + key] = "igemm"
    conv._choice[("dw3",) + key] = "igemm"
    try:
        y = m(x)
        dy = _cl(torch.randn_like(y.float()).bfloat16())
        y.backward(dy)
    finally:
        conv._choice.clear()
        conv._handoff.clear()
    w = m.weight._shadow.float().detach().requires_grad_(True)
    xr = x.detach().float().requires_grad_(True)
    ref = F.conv2d(xr, w, None, 2)
    ref.backward(dy.float())
    _close(y, ref)
    _close(x.grad, xr.grad)
    _close(m.weight.grad, w.grad)


@pytest.mark.parametrize("N,C,H,W,K", [(2, 64, 14, 14, 256), (3, 256, 9, 7, 64), (2, 128, 7, 7, 128)])
def test_conv1x1_implicit_gemm_matches_fp32(N, C, H, W, K):
    """The implicit-GEMM kernels with a 1x1 filter: forward (+ BN statistics),
    input gradient accumulated into an existing gradient, weight gradient into
    an fp32 buffer that already holds one -- against fp32 conv2d."""
    from distributed_tensorflow_example_amd.ops import conv

    g = torch.Generator(device="cuda").manual_seed(31 + C + K)
    x = _cl(torch.randn(N, C, H, W, device="cuda", generator=g).bfloat16())
    w = _cl((torch.randn(K, C, 1, 1, device="cuda", generator=g) * 0.05).bfloat16())
    assert conv.igemm1_ok(x, w)
    P = conv.conv3x3_stat_rows(x, 1)
    part = torch.full((2, P, K), float("nan"), device="cuda")
    y = conv.conv3x3(x, w, 1, stats=part)
    ref = F.conv2d(x.float(), w.float())
    _close(y, ref)
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, K)
    torch.testing.assert_close(part[0].sum(0), yf.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(part[1].sum(0), (yf * yf).sum(0), rtol=1e-4, atol=1e-2)
    dy = _cl(torch.randn(N, K, H, W, device="cuda", generator=g).bfloat16())
    prior = _cl(torch.randn(N, C, H, W, device="cuda", generator=g).bfloat16())
    dx = conv.conv3x3_dx(dy, w, x.shape, into=prior.clone())
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    F.conv2d(xr, wr).backward(dy.float())
    _close(dx, xr.grad + prior.float(), 2e-2)
    into = torch.randn(K, C, 1, 1, device="cuda", generator=g)
    base = into.clone()
    conv.conv3x3_dw(dy, x, 1, into=into)
    _close(into - base, wr.grad, 2e-3)


def test_shadow_conv1x1_on_igemm_trains_like_miopen(monkeypatch):
    """A 1x1 ShadowConv2d with every product forced onto the implicit GEMM
    (forward with the BN hand-off, input gradient, weight gradient) matches the
    MIOpen path of the same module."""
    from distributed_tensorflow_example_amd.ops import conv

    res = {}
    for eng in ("igemm", "miopen"):
        torch.manual_seed(2)
        m = conv.ShadowConv2d(128, 256, 1, 1, 0, bias=False).cuda().to(memory_format=torch.channels_last)
        conv.attach_shadows(m)
        x = _cl(torch.randn(2, 128, 16, 16, device="cuda").bfloat16()).requires_grad_(True)
        key = (tuple(x.shape), 256)
        conv._choice.clear()
        for role in ("fwd", "dx", "dw"):
            conv._choice[(role,) + key] = eng
        try:
            y = m(x)
            y.float().square().sum().backward()
        finally:
            conv._choice.clear()
            conv._handoff.clear()
        res[eng] = (y.float(), x.grad.float(), m.weight.grad.float())
    for a, b in zip(res["igemm"], res["miopen"]):
        _close(a, b, 2e-2)


def test_flipped_filter_cache_follows_optimizer_steps(monkeypatch):
    """The input gradient's flipped filters are cached per shadow version and
    re-flipped in one batched launch after a fused optimizer step: three
    momentum steps of two stacked convs (3x3 then 1x1, both on the implicit
    GEMM) match the uncached run, and the batched flip equals per-filter flips."""
    from distributed_tensorflow_example_amd import _native, optim
    from distributed_tensorflow_example_amd.ops import conv

    monkeypatch.setattr(conv, "_IGEMM", "always")
    N, C, H = 4, 64, 16
    key = ((N, C, H, H), C)
    monkeypatch.setattr(conv, "_choice", {("fwd",) + key: "igemm", ("dx",) + key: "igemm", ("dw",) + key: "igemm"})
    res = {}
    for cache in (True, False):
        monkeypatch.setattr(conv, "_FLIP_CACHE", cache)
        torch.manual_seed(4)
        net = torch.nn.Sequential(conv.ShadowConv2d(C, C, 3, 1, 1, bias=False),
                                  conv.ShadowConv2d(C, C, 1, bias=False)).cuda().to(memory_format=torch.channels_last)
        opt = optim.FusedMomentum(list(net.parameters()), 0.05, 0.9)
        conv.attach_shadows(net, opt)
        x = _cl(torch.randn(N, C, H, H, device="cuda").bfloat16()).requires_grad_(True)
        for _ in range(3):
            for p in net.parameters():
                p.grad = None
            x.grad = None
            net(x).float().square().mean().backward()
            opt.step()
        res[cache] = [p.detach().clone() for p in net.parameters()] + [x.grad.float()]
    for a, b in zip(res[True], res[False]):
        torch.testing.assert_close(a, b, rtol=0, atol=0)
    C_ = _native.load()
    ws = [_cl(torch.randn(96, 64, k, k, device="cuda").bfloat16()) for k in (1, 3, 3)]
    outs = [torch.empty((w.shape[1], w.shape[0], w.shape[2], w.shape[3]), device="cuda", dtype=torch.bfloat16,
                        memory_format=torch.channels_last) for w in ws]
    tab = torch.tensor([[w.data_ptr(), o.data_ptr(), w.shape[0], w.shape[1], w.shape[2]] for w, o in zip(ws, outs)],
                       dtype=torch.int64).cuda()
    tiles = torch.tensor([[i, rs, k0, c0] for i, w in enumerate(ws) for rs in range(w.shape[2] ** 2)
                          for k0 in range(0, w.shape[0], 64) for c0 in range(0, w.shape[1], 64)],
                         dtype=torch.int32).cuda()
    C_.conv_wflip_multi(tab, tiles)
    for w, o in zip(ws, outs):
        ref = torch.empty_like(o)
        C_.conv3x3_wflip(w, ref)
        assert torch.equal(o, ref)
