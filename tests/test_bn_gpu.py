"""Fused NHWC BatchNorm(+residual)(+ReLU) kernels vs a PyTorch fp32 reference."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


@pytest.mark.parametrize("C,HW", [(64, 56), (256, 14), (2048, 7), (24, 9), (4096, 3), (136, 5)])
@pytest.mark.parametrize("res,relu", [(False, True), (True, True), (False, False)])
def test_fused_bn_matches_reference(native, C, HW, res, relu):
    from distributed_tensorflow_example_amd.ops.bn import FusedBatchNorm2d

    torch.manual_seed(C + HW)
    N = 8
    x = (torch.randn(N, C, HW, HW) * 2 + 0.5).bfloat16().float()
    r = torch.randn(N, C, HW, HW).bfloat16().float() if res else None
    bn = FusedBatchNorm2d(C)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    ref_bn = torch.nn.BatchNorm2d(C)
    ref_bn.load_state_dict(bn.state_dict())
    xr = x.clone().requires_grad_()
    rr = r.clone().requires_grad_() if res else None
    yr = ref_bn(xr)
    if res:
        yr = yr + rr
    if relu:
        yr = F.relu(yr)
    dy = torch.randn_like(yr)
    yr.backward(dy)

    g = bn.cuda()
    xg = x.cuda().bfloat16().contiguous(memory_format=torch.channels_last).requires_grad_()
    rg = r.cuda().bfloat16().contiguous(memory_format=torch.channels_last).requires_grad_() if res else None
    y = g(xg, residual=rg, relu=relu)
    assert y.is_contiguous(memory_format=torch.channels_last)
    y.backward(dy.cuda().bfloat16().contiguous(memory_format=torch.channels_last))
    assert rel(y, yr) < 1e-2
    assert rel(xg.grad, xr.grad) < 3e-2
    if res:
        assert rel(rg.grad, rr.grad) < 2e-2
    assert rel(g.weight.grad, ref_bn.weight.grad) < 2e-2
    assert rel(g.bias.grad, ref_bn.bias.grad) < 2e-2
    assert rel(g.running_mean, ref_bn.running_mean) < 1e-3
    assert rel(g.running_var, ref_bn.running_var) < 1e-3
    assert int(g.state_dict()["num_batches_tracked"]) == int(ref_bn.num_batches_tracked) == 1


def test_resnet50_fused_bn_step_trains(native):
    from distributed_tensorflow_example_amd import optim
    from distributed_tensorflow_example_amd.models.resnet import resnet50, synthetic_imagenet_batch

    torch.manual_seed(0)
    m = resnet50(num_classes=10).cuda().to(memory_format=torch.channels_last)
    x, y = synthetic_imagenet_batch(16, "cuda", seed=1, size=64, num_classes=10)
    opt = optim.FusedMomentum(list(m.parameters()), 0.05, 0.9)
    losses = []
    for _ in range(12):
        for p in m.parameters():
            p.grad = None
        l = m.loss(x, y)
        l.backward()
        opt.step()
        losses.append(float(l))
    assert all(l == l for l in losses)          # no NaN
    assert losses[-1] < losses[0]


def test_bn_bwd_parts_fused_launch_many_shapes(native):
    """bn_bwd_parts (finalize + apply in one launch, blocks synchronised by a
    rotating pool of 256 monotonic counters) called 600 times with channel
    counts alternating 64 / 256 / 2048 -- every slot of the pool is reused with a
    different number of finalize blocks -- against the fp32 formula."""
    C_ = native
    cl = torch.channels_last
    cases = []
    for C in (64, 256, 2048):
        g = torch.Generator(device="cuda").manual_seed(C)
        N, H = 2, 8
        M = N * H * H
        x = torch.randn(N, C, H, H, device="cuda", generator=g).bfloat16().contiguous(memory_format=cl)
        gin = torch.randn(N, C, H, H, device="cuda", generator=g).bfloat16().contiguous(memory_format=cl)
        gamma = torch.rand(C, device="cuda", generator=g) + 0.5
        xf = x.float().permute(0, 2, 3, 1).reshape(M, C)
        gf = gin.float().permute(0, 2, 3, 1).reshape(M, C)
        mean, var = xf.mean(0), xf.var(0, unbiased=False)
        invstd = (var + 1e-5).rsqrt()
        stats = torch.cat([mean, invstd, gamma * invstd, -mean * gamma * invstd])
        xhat = (xf - mean) * invstd
        part = torch.stack([gf.sum(0), (gf * xhat).sum(0)]).reshape(2, 1, C).contiguous()
        dbeta, dgamma = gf.sum(0), (gf * xhat).sum(0)
        ref = gamma * invstd * (gf - dbeta / M - xhat * dgamma / M)
        cases.append((C, x, gin, gamma, stats, part, ref, dgamma, dbeta, M))
    for it in range(600):
        C, x, gin, gamma, stats, part, ref, rdg, rdb, M = cases[it % 3]
        dx = torch.empty_like(x)
        coef = torch.empty(3 * C, device="cuda")
        dg, db = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
        C_.bn_bwd_parts(gin, x, gamma, stats, part, 1, coef, dx, dg, db, False)
        if it % 97 == 0 or it >= 597:
            got = dx.float().permute(0, 2, 3, 1).reshape(M, C)
            torch.testing.assert_close(got, ref, rtol=2e-2, atol=2e-2)
            torch.testing.assert_close(dg, rdg, rtol=1e-4, atol=1e-3)
            torch.testing.assert_close(db, rdb, rtol=1e-4, atol=1e-3)
