"""Gradient sinks (ops.grad_sink): fused backward kernels accumulating weight
gradients straight into DDP bucket views must equal autograd's gradients."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


def _ddp(module):
    from distributed_tensorflow_example_amd.parallel.ddp import DistributedDataParallel
    from distributed_tensorflow_example_amd.parallel.world import World
    return DistributedDataParallel(module, World(device=torch.device("cuda", 0)), bucket_mb=1.0)


@pytest.mark.parametrize("k,stride", [(1, 1), (3, 2), (7, 2)])
def test_shadow_conv_sink_matches_autograd(native, k, stride):
    from distributed_tensorflow_example_amd.ops.conv import ShadowConv2d, attach_shadows
    torch.manual_seed(k)
    ref = torch.nn.Conv2d(32, 64, k, stride, k // 2, bias=False).cuda().to(memory_format=torch.channels_last)
    m = ShadowConv2d(32, 64, k, stride, k // 2, bias=False).cuda().to(memory_format=torch.channels_last)
    m.load_state_dict(ref.state_dict())
    attach_shadows(m)
    ddp = _ddp(m)
    ready = []
    ddp._launch = lambda bi: ready.append(bi)        # observe bucket completion
    x = torch.randn(4, 32, 20, 20, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    dy = torch.randn(4, 64, (20 + stride - 1) // stride, (20 + stride - 1) // stride, device="cuda").bfloat16()
    xr = x.clone().requires_grad_()
    with torch.autocast("cuda", torch.bfloat16):
        yr = ref(xr)
    yr.backward(dy.contiguous(memory_format=torch.channels_last))
    xs = x.clone().requires_grad_()
    for rep in range(2):                               # second pass accumulates
        y = ddp(xs)                                    # DDP.forward resets the ready counters
        y.backward(dy.contiguous(memory_format=torch.channels_last))
        assert rel(y, yr) < 1e-2
    assert m.weight.grad.data_ptr() == ddp.buckets[0].views[0].data_ptr()   # still the bucket view
    assert rel(m.weight.grad, 2 * ref.weight.grad) < 1e-2
    assert rel(xs.grad, 2 * xr.grad) < 1e-2
    assert ready == [0, 0]                             # the sink reported readiness each pass


def test_fused_bn_sink_accumulates_into_bucket(native):
    from distributed_tensorflow_example_amd.ops.bn import FusedBatchNorm2d
    torch.manual_seed(1)
    C = 64
    bn_a, bn_b = FusedBatchNorm2d(C).cuda(), FusedBatchNorm2d(C).cuda()
    with torch.no_grad():
        bn_a.weight.uniform_(0.5, 1.5)
    bn_b.load_state_dict(bn_a.state_dict())
    ddp = _ddp(bn_b)
    x = torch.randn(4, C, 10, 10, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    dy = torch.randn_like(x)
    for m in (bn_a, bn_b):
        xi = x.clone().requires_grad_()
        m(xi, relu=True).backward(dy)
    v = {id(p): t for p, t in zip(ddp.buckets[0].params, ddp.buckets[0].views)}
    for pa, pb in ((bn_a.weight, bn_b.weight), (bn_a.bias, bn_b.bias)):
        assert pb.grad.data_ptr() == v[id(pb)].data_ptr()
        assert rel(pb.grad, pa.grad) < 1e-5


def test_bert_gemm_sink_matches_plain(native):
    from distributed_tensorflow_example_amd.models.bert import BertConfig, BertForMLM, synthetic_mlm_batch
    c = BertConfig.tiny()
    c.dropout = c.attn_dropout = 0.0
    b = [t.cuda() for t in synthetic_mlm_batch(4, 64, c.vocab_size, "cpu", seed=3)]
    plain, sunk = BertForMLM(c, seed=7).cuda(), BertForMLM(c, seed=7).cuda()
    plain.attach_shadows()
    sunk.attach_shadows()
    ddp = _ddp(sunk)
    for _ in range(2):
        plain(*b).backward()
        ddp(*b).backward()                       # DDP.forward resets the per-bucket ready counts
        # every parameter reported ready exactly once (tied word embedding included)
        assert [bk.ready for bk in ddp.buckets] == [len(bk.params) for bk in ddp.buckets]
    gw = {id(w) for w in sunk.gemm_weights()}
    for (n, p1), p2 in zip(plain.named_parameters(), sunk.parameters()):
        assert rel(p2.grad, p1.grad) < 1e-3, n
        if id(p2) in gw:
            bi, idx = ddp._param_bucket[p2]
            assert p2.grad.data_ptr() == ddp.buckets[bi].views[idx].data_ptr()
