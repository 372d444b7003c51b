"""Fused transformer kernels vs PyTorch fp32 references, and a BERT step on GPU."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


@pytest.mark.parametrize("H", [256, 768, 1024, 3072])
@pytest.mark.parametrize("with_res", [True, False])
def test_bias_dropout_residual_layernorm_p0(native, H, with_res):
    from distributed_tensorflow_example_amd.ops import transformer as T
    torch.manual_seed(H)
    N = 333
    x = torch.randn(N, H).bfloat16()
    r = torch.randn(N, H).bfloat16() if with_res else None
    bias, g, b = torch.randn(H) * 0.1, 1 + 0.1 * torch.randn(H), 0.1 * torch.randn(H)
    xs = [t.float().clone().requires_grad_() if t is not None else None for t in (x, r)]
    ps = [t.clone().requires_grad_() for t in (bias, g, b)]
    ref = T.bias_dropout_residual_layernorm(xs[0], ps[0], xs[1], ps[1], ps[2], 0.0, 1e-12)
    dy = torch.randn(N, H)
    ref.backward(dy)
    xg = x.cuda().requires_grad_()
    rg = r.cuda().requires_grad_() if r is not None else None
    pg = [t.cuda().requires_grad_() for t in (bias, g, b)]
    out = T.bias_dropout_residual_layernorm(xg, pg[0], rg, pg[1], pg[2], 0.0, 1e-12)
    out.backward(dy.cuda().bfloat16())
    assert rel(out, ref) < 1e-2
    assert rel(xg.grad, xs[0].grad) < 2e-2
    if r is not None:
        assert rel(rg.grad, xs[1].grad) < 2e-2
    for a, b_ in zip(pg, ps):
        assert rel(a.grad, b_.grad) < 2e-2


def test_bdrln_dropout_mask_consistency(native):
    """With p > 0: kept fraction ~ 1-p and backward uses exactly the forward mask."""
    from distributed_tensorflow_example_amd.ops import transformer as T
    N, H, p = 512, 768, 0.25
    x = torch.randn(N, H, device="cuda").bfloat16().requires_grad_()
    bias = torch.zeros(H, device="cuda", requires_grad=True)
    g, b = torch.ones(H, device="cuda"), torch.zeros(H, device="cuda")
    out = T.bias_dropout_residual_layernorm(x, bias, None, g, b, p, 1e-12)
    out.backward(torch.ones_like(out))
    # dropped elements receive exactly zero gradient
    zero_grad = (x.grad == 0).float().mean().item()
    assert abs(zero_grad - p) < 0.02


@pytest.mark.parametrize("N", [512, 333])
def test_bdrln_forward_mask_is_backward_mask(native, N):
    """The dropped elements of the forward's saved s (bdrln_fwd, 16-byte half-wave
    rows) are exactly the ones ln_bwd's dropout-branch gradient zeroes (same
    element indices), odd row counts included."""
    from distributed_tensorflow_example_amd.ops import transformer as T
    C = T._C()
    H, p, seed = 768, 0.25, -(1 << 63) + 977
    torch.manual_seed(5)
    x = torch.randn(N, H, device="cuda").bfloat16() + 4.0     # no exact zeros before dropout
    bias, g, b = torch.zeros(H, device="cuda"), torch.ones(H, device="cuda"), torch.zeros(H, device="cuda")
    y, s = torch.empty_like(x), torch.empty_like(x)
    mean, rstd = torch.empty(N, device="cuda"), torch.empty(N, device="cuda")
    C.bdrln_fwd(x, bias, None, g, b, y, s, mean, rstd, 1e-12, p, seed)
    dy = torch.randn_like(x)
    ds, dxb = torch.empty_like(x), torch.empty_like(x)
    dg, db, dbias = (torch.empty(H, device="cuda") for _ in range(3))
    C.ln_bwd(dy, s, mean, rstd, g, ds, dxb, T._ln_part(N, H, x.device), dg, db, dbias, p, seed, False)
    dropped_f, dropped_b = s == 0, (dxb == 0) & (ds != 0)
    assert abs(float(dropped_f.float().mean()) - p) < 0.02
    assert int((dropped_f & (ds != 0) != dropped_b).sum()) == 0
    ref = torch.nn.functional.layer_norm(s.float(), (H,), eps=1e-12)
    assert rel(y, ref) < 1e-2


def test_layernorm_dropout_embeddings(native):
    from distributed_tensorflow_example_amd.ops import transformer as T
    N, H = 200, 768
    x = torch.randn(N, H)
    g, b = 1 + 0.1 * torch.randn(H), 0.1 * torch.randn(H)
    xr, gr, br = x.clone().requires_grad_(), g.clone().requires_grad_(), b.clone().requires_grad_()
    ref = T.layernorm_dropout(xr, gr, br, 0.0)
    dy = torch.randn(N, H)
    ref.backward(dy)
    xg, gg, bg = x.cuda().requires_grad_(), g.cuda().requires_grad_(), b.cuda().requires_grad_()
    out = T.layernorm_dropout(xg, gg, bg, 0.0)
    out.backward(dy.cuda().bfloat16())
    assert rel(out, ref) < 1e-2 and rel(xg.grad, xr.grad) < 2e-2 and rel(gg.grad, gr.grad) < 2e-2


@pytest.mark.parametrize("N,H", [(128, 3072), (1000, 768), (7, 1024)])
def test_bias_gelu(native, N, H):
    from distributed_tensorflow_example_amd.ops import transformer as T
    x = torch.randn(N, H).bfloat16()
    bias = torch.randn(H) * 0.2
    xr, br = x.float().requires_grad_(), bias.clone().requires_grad_()
    ref = T.bias_gelu(xr, br)
    dy = torch.randn(N, H)
    ref.backward(dy)
    xg, bg = x.cuda().requires_grad_(), bias.cuda().requires_grad_()
    out = T.bias_gelu(xg, bg)
    out.backward(dy.cuda().bfloat16())
    assert rel(out, ref) < 1e-2 and rel(xg.grad, xr.grad) < 2e-2 and rel(bg.grad, br.grad) < 2e-2


@pytest.mark.parametrize("S", [64, 128, 384, 512])
def test_attention_softmax(native, S):
    from distributed_tensorflow_example_amd.ops import transformer as T
    B, Hh = 3, 4
    sc = (torch.randn(B, Hh, S, S) * 4).bfloat16()
    mask = torch.zeros(B, S)
    mask[1, S // 2:] = -10000.0
    scr = sc.float().requires_grad_()
    ref = T.attention_softmax(scr, mask, 1 / 8, 0.0)
    dp = torch.randn_like(ref)
    ref.backward(dp)
    sg = sc.cuda().requires_grad_()
    out = T.attention_softmax(sg, mask.cuda(), 1 / 8, 0.0)
    out.backward(dp.cuda().bfloat16())
    assert rel(out, ref) < 1e-2
    assert rel(sg.grad, scr.grad) < 3e-2
    assert float(out[1, :, :, S // 2:].float().abs().max()) < 1e-6       # masked keys get ~0 prob


def test_attention_softmax_dropout_stats(native):
    from distributed_tensorflow_example_amd.ops import transformer as T
    sc = torch.zeros(2, 2, 128, 128, device="cuda", dtype=torch.bfloat16)
    out = T.attention_softmax(sc, None, 1.0, 0.1)
    kept = (out > 0).float().mean().item()
    assert abs(kept - 0.9) < 0.01
    assert abs(out.float().sum(-1).mean().item() - 1.0) < 0.02      # inverted dropout keeps the expectation


def test_bert_tiny_gpu_matches_cpu_and_trains(native):
    from distributed_tensorflow_example_amd import optim
    from distributed_tensorflow_example_amd.models.bert import BertConfig, BertForMLM, synthetic_mlm_batch

    c = BertConfig.tiny()
    c.dropout = c.attn_dropout = 0.0
    cpu = BertForMLM(c, seed=3)
    gpu = BertForMLM(c, seed=3).cuda()
    b = synthetic_mlm_batch(8, 128, c.vocab_size, "cpu", seed=1)
    lc = cpu(*b)
    lg = gpu(*[t.cuda() for t in b])
    assert abs(float(lc) - float(lg)) < 0.05 * abs(float(lc))
    lc.backward()
    lg.backward()
    for (n, pc), pg in zip(cpu.named_parameters(), gpu.parameters()):
        if pc.grad is not None and pc.grad.norm() > 1e-6:
            assert rel(pg.grad, pc.grad) < 0.1, n
    c.dropout = c.attn_dropout = 0.1
    m = BertForMLM(c, seed=4).cuda()
    opt = optim.FusedAdamW(list(m.parameters()), 1e-3, weight_decay=0.01)
    losses = []
    for i in range(30):
        for p in m.parameters():
            p.grad = None
        l = m(*[t.cuda() for t in b])
        l.backward()
        opt.step()
        losses.append(float(l))
    assert losses[-1] < losses[0] - 1.0


def test_bert_bf16_shadow_weights_match_casts(native):
    from distributed_tensorflow_example_amd import optim
    from distributed_tensorflow_example_amd.models.bert import BertConfig, BertForMLM, synthetic_mlm_batch

    c = BertConfig.tiny()
    c.dropout = c.attn_dropout = 0.0
    b = [t.cuda() for t in synthetic_mlm_batch(8, 128, c.vocab_size, "cpu", seed=2)]
    plain, shad = BertForMLM(c, seed=5).cuda(), BertForMLM(c, seed=5).cuda()
    o1 = optim.FusedAdamW(list(plain.parameters()), 1e-3)
    o2 = optim.FusedAdamW(list(shad.parameters()), 1e-3)
    shad.attach_shadows(o2)
    for _ in range(3):
        for m, o in ((plain, o1), (shad, o2)):
            for p in m.parameters():
                p.grad = None
            m(*b).backward()
            o.step()
    # Adam moves every parameter by ~lr per step whatever the gradient size, so
    # near-zero params (LN betas, biases) can differ by O(lr) where a tiny bf16
    # gradient difference flips a sign; the GEMM weights must agree tightly
    gw = {id(w) for w in shad.gemm_weights()}
    for (n, p1), p2 in zip(plain.named_parameters(), shad.parameters()):
        if id(p2) in gw:
            assert rel(p1, p2) < 2e-3, n
        else:
            assert float((p1 - p2).abs().max()) < 6e-3, n
    for w in shad.gemm_weights():
        assert torch.equal(w._shadow, w.detach().bfloat16())


def test_bert_residual_grad_slot_matches_autograd_add(native):
    """Shadow-weight BERT folds LN residual gradients into the dX GEMMs
    (GradSlot); one backward must give the same gradients as the plain model,
    whose residual gradients meet in autograd's add."""
    from distributed_tensorflow_example_amd.models.bert import BertConfig, BertForMLM, synthetic_mlm_batch
    from distributed_tensorflow_example_amd.ops import transformer as T

    c = BertConfig.tiny()
    c.dropout = c.attn_dropout = 0.0
    b = [t.cuda() for t in synthetic_mlm_batch(8, 128, c.vocab_size, "cpu", seed=4)]
    plain, shad = BertForMLM(c, seed=6).cuda(), BertForMLM(c, seed=6).cuda()
    shad.attach_shadows()
    taken = []
    orig = T.GradSlot.take
    T.GradSlot.take = lambda self: taken.append(self.g is not None) or orig(self)
    try:
        plain(*b).backward()
        shad(*b).backward()
    finally:
        T.GradSlot.take = orig
    assert taken and all(taken), taken          # every slot was filled by its LN before the GEMM ran
    for (n, p1), p2 in zip(plain.named_parameters(), shad.parameters()):
        if p1.grad is not None and p1.grad.norm() > 1e-6:
            assert rel(p2.grad, p1.grad) < 2e-2, n


def _unfused_attention(qkv, bias, mask, nh, scale, p):
    """The model's pre-fusion GPU path: bias add, batched GEMMs, softmax kernel."""
    from distributed_tensorflow_example_amd.ops import transformer as T
    B, S, H3 = qkv.shape
    d = H3 // (3 * nh)
    x = (qkv + bias.to(qkv.dtype)).view(B, S, 3, nh, d)
    q, k, v = x[:, :, 0].permute(0, 2, 1, 3), x[:, :, 1].permute(0, 2, 3, 1), x[:, :, 2].permute(0, 2, 1, 3)
    probs = T.attention_softmax(torch.matmul(q, k), mask, scale, p)
    return torch.matmul(probs.to(v.dtype), v).permute(0, 2, 1, 3).reshape(B, S, nh * d)


@pytest.mark.parametrize("S", [32, 64, 128, 192, 256])
def test_fused_attention_matches_fp32_reference(native, S):
    from distributed_tensorflow_example_amd.ops import transformer as T
    assert T.attention_supported(S, 64)
    torch.manual_seed(S)
    B, nh = 3, 4
    qkv = (torch.randn(B, S, 3 * nh * 64) * 2).bfloat16()
    bias = torch.randn(3 * nh * 64) * 0.5
    mask = torch.zeros(B, S)
    mask[1, S // 2:] = -10000.0
    mask[2, S - 5:] = -10000.0
    scale = 1 / 8
    xr, br = qkv.float().requires_grad_(), bias.clone().requires_grad_()
    ref = T.attention_reference(xr, br, mask, nh, scale)
    dy = torch.randn_like(ref)
    ref.backward(dy)
    xg, bg = qkv.cuda().requires_grad_(), bias.cuda().requires_grad_()
    out = T.fused_attention(xg, bg, mask.cuda(), nh, scale)
    out.backward(dy.cuda().bfloat16())
    assert out.shape == (B, S, nh * 64) and out.dtype == torch.bfloat16
    assert rel(out, ref) < 1e-2
    assert rel(xg.grad, xr.grad) < 3e-2
    for part in range(3):                          # q, k, v blocks separately
        sl = slice(part * nh * 64, (part + 1) * nh * 64)
        assert rel(xg.grad[..., sl], xr.grad[..., sl]) < 3e-2, part
    assert rel(bg.grad, br.grad) < 3e-2
    # the in-kernel bias partials sum the fp32 values dqkv was rounded from
    assert rel(bg.grad, xg.grad.float().sum((0, 1))) < 5e-3


def test_fused_attention_dropout_matches_unfused_kernel_path(native):
    """Same seed -> the fused kernel drops exactly the elements the softmax kernel drops."""
    from distributed_tensorflow_example_amd.ops import transformer as T
    torch.manual_seed(0)
    B, S, nh, p = 2, 128, 4, 0.2
    qkv = torch.randn(B, S, 3 * nh * 64, device="cuda").bfloat16()
    bias = torch.randn(3 * nh * 64, device="cuda") * 0.3
    mask = torch.zeros(B, S, device="cuda")
    mask[0, 100:] = -10000.0
    dy = torch.randn(B, S, nh * 64, device="cuda").bfloat16()
    outs = []
    for fused in (True, False):
        T.set_dropout_seed(1234)
        x, b = qkv.clone().requires_grad_(), bias.clone().requires_grad_()
        o = T.fused_attention(x, b, mask, nh, 0.125, p) if fused else _unfused_attention(x, b, mask, nh, 0.125, p)
        o.backward(dy)
        outs.append((o, x.grad, b.grad))
    (o1, g1, b1), (o2, g2, b2) = outs
    assert rel(o1, o2) < 2e-2
    assert rel(g1, g2) < 4e-2
    assert rel(b1, b2) < 4e-2


@pytest.mark.parametrize("N,H", [(16384, 2304), (1000, 768), (37, 64), (300, 520)])
def test_colsum_bf16_matches_torch(native, N, H):
    x = torch.randn(N, H, device="cuda").bfloat16()
    part = torch.empty(max(1, min(256, N // 64)) * H, device="cuda")
    out = torch.full((H,), 0.5, device="cuda")
    native.colsum_bf16(x, part, out, accumulate=True)
    ref = x.float().sum(0) + 0.5
    assert torch.allclose(out, ref, rtol=1e-4, atol=1e-3 * (N ** 0.5))
    native.colsum_bf16(x, part, out, accumulate=False)
    assert torch.allclose(out, ref - 0.5, rtol=1e-4, atol=1e-3 * (N ** 0.5))


@pytest.mark.parametrize("S,n", [(1, 4), (3, 1001), (4, 768 * 3072), (16, 2304 * 768)])
def test_slab_sum_matches_torch(native, S, n):
    slabs = torch.randn(S, n, device="cuda")
    out = torch.randn(n, device="cuda")
    ref = out + slabs.sum(0)
    native.slab_sum(slabs, out, accumulate=True)
    assert torch.allclose(out, ref, rtol=1e-5, atol=1e-5)
    native.slab_sum(slabs, out, accumulate=False)
    assert torch.allclose(out, slabs.sum(0), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("H", [256, 768])
def test_bert_embed_fused_matches_reference(native, H):
    """The fused embedding block (gather word / type / position rows + LayerNorm,
    one kernel; position and 2-row type gradients in one pass, word rows by the
    sorted scatter) against the fp32 composition: output and every gradient."""
    from distributed_tensorflow_example_amd.ops import transformer as T
    torch.manual_seed(H)
    B, S, V = 4, 16, 1000
    word, typ, pos = torch.randn(V, H) * 0.1, torch.randn(2, H) * 0.1, torch.randn(64, H) * 0.1
    gamma, beta = 1 + 0.1 * torch.randn(H), 0.1 * torch.randn(H)
    ids = torch.randint(0, V, (B, S))
    ids[0, :4] = 7                                 # repeated rows in the scatter
    tt = torch.randint(0, 2, (B, S))
    ref_p = [t.clone().requires_grad_() for t in (word, typ, pos, gamma, beta)]
    x = ref_p[0][ids] + ref_p[1][tt] + ref_p[2][:S].unsqueeze(0)
    ref = torch.nn.functional.layer_norm(x, (H,), ref_p[3], ref_p[4], 1e-12)
    gy = torch.randn_like(ref)
    ref.backward(gy)
    got_p = [t.cuda().requires_grad_() for t in (word, typ, pos, gamma, beta)]
    out = T.bert_embed(*got_p, ids.cuda(), tt.cuda(), 0.0, 1e-12, True)
    assert out.dtype == torch.bfloat16 and out.shape == (B, S, H)
    out.backward(gy.cuda().bfloat16())
    assert (out.float().cpu() - ref.detach()).abs().max() < 3e-2
    for g, r in zip(got_p, ref_p):
        err = float((g.grad.float().cpu() - r.grad).norm() / r.grad.norm().clamp_min(1e-12))
        assert err < 2e-2, err


def test_bert_embed_fused_dropout_consistent(native):
    """p > 0: the forward's dropped elements are exactly the ones the backward
    masks (same hash), and about p of them are dropped."""
    from distributed_tensorflow_example_amd.ops import transformer as T
    torch.manual_seed(1)
    B, S, H, V, p = 8, 32, 256, 500, 0.25
    ps = [t.cuda().requires_grad_() for t in (torch.randn(V, H), torch.randn(2, H), torch.randn(S, H),
                                             torch.ones(H), torch.zeros(H))]
    ids, tt = torch.randint(0, V, (B, S)).cuda(), torch.randint(0, 2, (B, S)).cuda()
    out = T.bert_embed(*ps, ids, tt, p, 1e-12, True)
    dropped = out.float() == 0
    frac = float(dropped.float().mean())
    assert abs(frac - p) < 0.03, frac
    out.float().sum().backward()
    assert torch.isfinite(ps[0].grad).all() and torch.isfinite(ps[2].grad).all()
    # beta's gradient counts the kept elements only (each kept output scales by
    # 1/(1-p); the backward's dropout rescale is bf16: 1.3359 for 1/0.75)
    kept = (~dropped).float().sum(dim=(0, 1)) / (1 - p)
    assert torch.allclose(ps[4].grad, kept, rtol=5e-3, atol=1e-2)


def test_bert_tied_word_grad_fused_matches_composed(native, monkeypatch):
    """BertForMLM's tied word table: the fused embedding's backward scatters its
    rows straight into the MLM decoder's dW (no zeroed table, no autograd add);
    the summed gradient must equal the composed path's (DTF_BERT_EMB_FUSED=0),
    over two steps (a stale decoder dW from an earlier step is never reused)."""
    from distributed_tensorflow_example_amd.models import bert
    c = bert.BertConfig.tiny()
    c.dropout = 0.0
    B, S = 4, 32
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(0, c.vocab_size, (B, S), generator=g).cuda()
    tt = torch.randint(0, 2, (B, S), generator=g).cuda()
    mask = torch.ones(B, S, dtype=torch.int64).cuda()
    pos = torch.arange(0, B * S, 5).cuda()
    lab = torch.randint(0, c.vocab_size, (pos.numel(),), generator=g).cuda()

    def grads(fused):
        monkeypatch.setenv("DTF_BERT_EMB_FUSED", "1" if fused else "0")
        m = bert.BertForMLM(c, seed=0).cuda()
        m.attach_shadows()
        out = []
        for _ in range(2):
            m.zero_grad(set_to_none=True)
            m(ids, tt, mask, pos, lab).backward()
            out.append([p.grad.detach().clone() for p in (m.word, m.pos, m.typ)])
        if fused:
            assert getattr(m.word, "_dtf_tied_dw", "absent") is None   # parked, then consumed
        return out

    for a, b in zip(grads(True), grads(False)):
        for x, y in zip(a, b):
            err = float((x - y).norm() / y.norm().clamp_min(1e-12))
            assert err < 2e-2, err
