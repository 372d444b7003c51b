"""Autograd wrappers for the fused transformer kernels (csrc/kernels/transformer.hip).

GPU tensors run the HIP kernels (bf16 activations, fp32 statistics and
parameters); CPU tensors run an equivalent PyTorch formulation -- the
numerics oracle for the GPU tests (dropout p = 0 there; the GPU dropout mask
is a counter hash of (seed, element index) regenerated in backward).
"""
from __future__ import annotations

import itertools
import os
import math
from typing import Optional

import torch

from .. import _native

_seed_counter = itertools.count(1)
_BASE_SEED = 0x5EED


# bit 63 of a dropout seed selects the 32-bit hash in the kernels (csrc/kernels/
# common.h hash32); DTF_DROPOUT_HASH=64 keeps the splitmix64 one.  Seeds cross
# into C++ as int64: bit 63 set = a negative Python int (same bits).
_FAST_HASH = -(1 << 63) if os.environ.get("DTF_DROPOUT_HASH", "32") != "64" else 0


# qkv bias gradient from the attention backward kernels' own partial sums (1), or
# a separate column-sum pass over dqkv (0, A/B)
_ATTN_BIAS_PARTIALS = os.environ.get("DTF_ATTN_BIAS_PARTIALS", "1") != "0"


def next_seed() -> int:
    return ((_BASE_SEED * 1000003 + next(_seed_counter) * 0x9E3779B1) & ((1 << 62) - 1)) + _FAST_HASH


def set_dropout_seed(seed: int):
    global _seed_counter, _BASE_SEED
    _BASE_SEED = int(seed)
    _seed_counter = itertools.count(1)


from . import grad_sink  # noqa: E402


def _C():
    return _native.load()


def _ln_part(N: int, H: int, device) -> torch.Tensor:
    # 4 blocks per CU (16 waves) with ~4 rows per wave: at 1 block per CU the
    # per-row load -> reduce -> store latency chain ran 3x off HBM bandwidth
    grid = max(1, min(1024, (N + 15) // 16))     # one partial row per block
    return torch.empty(3 * grid * H, dtype=torch.float32, device=device)


# ---------------------------------------------------------------- bias + dropout + residual + LN
class GradSlot:
    """Hands the residual-branch gradient of a post-LN epilogue to the GEMM
    whose input is the same activation (BERT: a layer's input feeds both the
    QKV projection and LN1's residual; LN1's output feeds both W1 and LN2's
    residual).  The LN backward parks ds here instead of returning it, and the
    GEMM backward folds it in as the beta = 1 term of its dX GEMM -- one fewer
    full-activation bf16 add per residual per step.  The LN backward always
    runs first (the GEMM's upstream gradient depends on it); if the GEMM's
    backward somehow ran first (`consumed`), the LN returns ds normally."""

    __slots__ = ("g", "consumed")

    def __init__(self):
        self.g = None
        self.consumed = False

    def take(self):
        g, self.g, self.consumed = self.g, None, True
        return g


class _BDRLN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, res, gamma, beta, p, eps, slot=None):
        C = _C()
        H = x.shape[-1]
        x2 = x.reshape(-1, H).contiguous()
        N = x2.shape[0]
        y = torch.empty_like(x2)
        s = torch.empty_like(x2)
        mean = torch.empty(N, dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        seed = next_seed() if p > 0 else 0
        r2 = res.reshape(-1, H).contiguous() if res is not None else None
        C.bdrln_fwd(x2, bias, r2, gamma, beta, y, s, mean, rstd, eps, p, seed)
        ctx.save_for_backward(s, mean, rstd, gamma)
        ctx.params = (gamma, beta, bias)   # for sinking dgamma/dbeta/dbias into .grad
        ctx.p, ctx.seed, ctx.has_res, ctx.shape = p, seed, res is not None, x.shape
        ctx.slot = slot if res is not None else None
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        C = _C()
        s, mean, rstd, gamma = ctx.saved_tensors
        H = s.shape[-1]
        dy2 = dy.reshape(-1, H).to(torch.bfloat16).contiguous()
        N = dy2.shape[0]
        ds = torch.empty_like(dy2)
        dxb = torch.empty_like(dy2)
        pg, pb, px = ctx.params
        sink = grad_sink.all_enabled(pg, pb, px)
        if sink:   # accumulate straight into the DDP bucket views (no AccumulateGrad adds)
            dgamma, dbeta, dbias = grad_sink.target(pg), grad_sink.target(pb), grad_sink.target(px)
        else:
            dgamma = torch.empty(H, dtype=torch.float32, device=dy.device)
            dbeta = torch.empty_like(dgamma)
            dbias = torch.empty_like(dgamma)
        C.ln_bwd(dy2, s, mean, rstd, gamma, ds, dxb, _ln_part(N, H, dy.device), dgamma, dbeta, dbias, ctx.p, ctx.seed,
                 accumulate=sink)
        dres = ds.view(ctx.shape) if ctx.has_res else None
        if dres is not None and ctx.slot is not None and not ctx.slot.consumed:
            ctx.slot.g, dres = dres, None   # folded into the consuming GEMM's dX
        if sink:
            for q in (pg, pb, px):
                grad_sink.done(q)
            return dxb.view(ctx.shape), None, dres, None, None, None, None, None
        return dxb.view(ctx.shape), dbias, dres, dgamma, dbeta, None, None, None


def bias_dropout_residual_layernorm(x, bias, residual, gamma, beta, p: float = 0.0, eps: float = 1e-12,
                                   training: bool = True, residual_slot: "GradSlot" = None):
    """LayerNorm(dropout(x + bias) + residual) -- the post-sublayer epilogue.

    `residual_slot`: see GradSlot (GPU path, bf16 residual only)."""
    p = p if training else 0.0
    if not x.is_cuda:
        t = x.float() + bias
        if p > 0:
            t = torch.nn.functional.dropout(t, p, True)
        if residual is not None:
            t = t + residual.float()
        return torch.nn.functional.layer_norm(t, (t.shape[-1],), gamma, beta, eps)
    if residual is not None and residual.dtype != torch.bfloat16:
        residual_slot = None      # the cast node, not the GEMM input, would receive the gradient
    return _BDRLN.apply(x.to(torch.bfloat16), bias, None if residual is None else residual.to(torch.bfloat16),
                        gamma, beta, float(p), float(eps), residual_slot)


class _EmbLN(torch.autograd.Function):
    """y = dropout(LayerNorm(x)); x fp32 (summed embeddings), y bf16."""

    @staticmethod
    def forward(ctx, x, gamma, beta, p, eps):
        C = _C()
        H = x.shape[-1]
        x2 = x.reshape(-1, H).contiguous().float()
        N = x2.shape[0]
        y = torch.empty(x2.shape, dtype=torch.bfloat16, device=x.device)
        s = torch.empty_like(y)
        mean = torch.empty(N, dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        seed = next_seed() if p > 0 else 0
        C.ln_fwd_f32in(x2, gamma, beta, y, s, mean, rstd, eps, p, seed)
        ctx.save_for_backward(s, mean, rstd, gamma)
        ctx.params = (gamma, beta)
        ctx.p, ctx.seed, ctx.shape = p, seed, x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        C = _C()
        s, mean, rstd, gamma = ctx.saved_tensors
        H = s.shape[-1]
        dy2 = dy.reshape(-1, H).to(torch.bfloat16).contiguous()
        if ctx.p > 0:
            dyd = torch.empty_like(dy2)
            C.dropout_bf16(dy2, dyd, ctx.p, ctx.seed)
            dy2 = dyd
        N = dy2.shape[0]
        ds = torch.empty_like(dy2)
        pg, pb = ctx.params
        sink = grad_sink.all_enabled(pg, pb)
        if sink:
            dgamma, dbeta = grad_sink.target(pg), grad_sink.target(pb)
        else:
            dgamma = torch.empty(H, dtype=torch.float32, device=dy.device)
            dbeta = torch.empty_like(dgamma)
        C.ln_bwd(dy2, s, mean, rstd, gamma, ds, None, _ln_part(N, H, dy.device), dgamma, dbeta, None, 0.0, 0,
                 accumulate=sink)
        if sink:
            grad_sink.done(pg)
            grad_sink.done(pb)
            return ds.float().view(ctx.shape), None, None, None, None
        return ds.float().view(ctx.shape), dgamma, dbeta, None, None


class _BertEmbed(torch.autograd.Function):
    """y = dropout(LayerNorm(word[ids] + typ[tt] + pos[:S])) (bf16) in one kernel
    that gathers the fp32 rows itself (csrc/kernels/transformer.hip emb_ln_fwd);
    backward: ln_bwd -> ds, then the position and 2-row token-type gradients
    from ds in one pass (emb_bwd_aux + one finishing colsum) and the word rows
    through the sorted-segment scatter.  Replaces the fp32 [tokens, H] sum, its
    lerp / adds and torch's reductions over the batch."""

    @staticmethod
    def forward(ctx, word, typ, pos, gamma, beta, ids, tt, p, eps):
        C = _C()
        B, S = ids.shape
        H = word.shape[-1]
        N = B * S
        y = torch.empty((N, H), dtype=torch.bfloat16, device=word.device)
        s = torch.empty_like(y)
        mean = torch.empty(N, dtype=torch.float32, device=word.device)
        rstd = torch.empty_like(mean)
        seed = next_seed() if p > 0 else 0
        idf, ttf = ids.reshape(-1).contiguous(), tt.reshape(-1).contiguous()
        C.emb_ln_fwd(word, idf, typ, ttf, pos, S, gamma, beta, y, s, mean, rstd, eps, p, seed)
        ctx.save_for_backward(s, mean, rstd, gamma, idf, ttf)
        ctx.params = (gamma, beta, pos, typ)
        ctx.p, ctx.seed, ctx.B, ctx.S, ctx.wshape = p, seed, B, S, word.shape
        # tied word table (MLM decoder): this forward's token, see backward
        ctx.word = word
        ctx.epoch = word._dtf_tied_epoch = object() if getattr(word, "_dtf_tied", False) else None
        return y.view(B, S, H)

    @staticmethod
    def backward(ctx, dy):
        from . import _bag_plan
        C = _C()
        s, mean, rstd, gamma, idf, ttf = ctx.saved_tensors
        H = s.shape[-1]
        dy2 = dy.reshape(-1, H).to(torch.bfloat16).contiguous()
        if ctx.p > 0:
            dyd = torch.empty_like(dy2)
            C.dropout_bf16(dy2, dyd, ctx.p, ctx.seed)
            dy2 = dyd
        N = dy2.shape[0]
        ds = torch.empty_like(dy2)
        pg, pb, ppos, ptyp = ctx.params
        sink = grad_sink.all_enabled(pg, pb)
        if sink:
            dgamma, dbeta = grad_sink.target(pg), grad_sink.target(pb)
        else:
            dgamma = torch.empty(H, dtype=torch.float32, device=dy.device)
            dbeta = torch.empty_like(dgamma)
        C.ln_bwd(dy2, s, mean, rstd, gamma, ds, None, _ln_part(N, H, dy.device), dgamma, dbeta, None, 0.0, 0,
                 accumulate=sink)
        # position + token-type gradients: one pass over ds
        sink2 = grad_sink.all_enabled(ppos, ptyp)
        if sink2:
            dpos, dtyp = grad_sink.target(ppos), grad_sink.target(ptyp)
        else:
            dpos = torch.zeros_like(ppos)
            dtyp = torch.empty_like(ptyp)
        part = torch.empty(2 * ctx.S * H, dtype=torch.float32, device=dy.device)
        C.emb_bwd_aux(ds, ttf, ctx.S, dpos, dtyp, part, sink2)
        # word rows: the sorted-segment scatter (one bag per token).  A tied table
        # whose decoder gradient of THIS forward is parked on the parameter takes
        # the rows straight into that tensor (autograd then has nothing to add)
        gw, ret = None, True
        if ctx.epoch is not None:
            tied = getattr(ctx.word, "_dtf_tied_dw", None)
            ctx.word._dtf_tied_dw = None
            if (tied is not None and tied[0] is ctx.epoch and tied[1].dtype == torch.float32
                    and tied[1].shape == ctx.wshape and tied[1].is_contiguous()):
                gw, ret = tied[1], False
        if gw is None:
            gw = torch.zeros(ctx.wshape, dtype=torch.float32, device=dy.device)
        offs = _identity_offsets(N, dy.device)
        rows, occ, bag_of = _bag_plan(idf, offs)
        C.embedding_bag_bwd_sorted(gw, rows, occ, bag_of, None, ds.float())
        if not ret:
            gw = None
        if sink:
            grad_sink.done(pg)
            grad_sink.done(pb)
            dgamma = dbeta = None
        if sink2:
            grad_sink.done(ppos)
            grad_sink.done(ptyp)
            dpos = dtyp = None
        return gw, dtyp, dpos, dgamma, dbeta, None, None, None, None


_IDOFFS: dict = {}


def _identity_offsets(n: int, device) -> torch.Tensor:
    """arange(n + 1) on `device`, cached (one bag per token)."""
    key = (n, str(device))
    t = _IDOFFS.get(key)
    if t is None:
        t = _IDOFFS[key] = torch.arange(n + 1, device=device)
    return t


def bert_embed(word, typ, pos, gamma, beta, ids, tt, p: float = 0.0, eps: float = 1e-12, training: bool = True):
    """dropout(LayerNorm(word[ids] + typ[tt] + pos[:S])) for [B, S] ids; bf16 out
    on the GPU (fused), the plain composition elsewhere."""
    p = p if training else 0.0
    S = ids.shape[1]
    if (not word.is_cuda or typ.shape[0] != 2 or word.shape[-1] % 256 or word.shape[-1] > 1024
            or ids.dtype != torch.int64 or tt.dtype != torch.int64):
        x = word[ids] + typ[tt] + pos[:S].unsqueeze(0)
        return layernorm_dropout(x, gamma, beta, p, eps, training)
    return _BertEmbed.apply(word, typ, pos, gamma, beta, ids, tt, float(p), float(eps))


def layernorm_dropout(x, gamma, beta, p: float = 0.0, eps: float = 1e-12, training: bool = True):
    p = p if training else 0.0
    if not x.is_cuda:
        y = torch.nn.functional.layer_norm(x.float(), (x.shape[-1],), gamma, beta, eps)
        return torch.nn.functional.dropout(y, p, True) if p > 0 else y
    return _EmbLN.apply(x, gamma, beta, float(p), float(eps))


# ---------------------------------------------------------------- bias + GELU
class _BiasGelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias):
        C = _C()
        x2 = x.contiguous()
        y = torch.empty_like(x2)
        C.bias_gelu_fwd(x2, bias, y)
        ctx.save_for_backward(x2, bias)
        ctx.bias_param = bias
        return y

    @staticmethod
    def backward(ctx, dy):
        C = _C()
        x, bias = ctx.saved_tensors
        H = x.shape[-1]
        N = x.numel() // H
        dx = torch.empty_like(x)
        slices = max(1, min(512, N // 32))        # >= 32 rows per thread, ~1.5k blocks at BERT-base
        part = torch.empty(slices * H, dtype=torch.float32, device=x.device)
        pb = ctx.bias_param
        sink = grad_sink.all_enabled(pb)
        dbias = grad_sink.target(pb) if sink else torch.empty(H, dtype=torch.float32, device=x.device)
        C.bias_gelu_bwd(dy.to(torch.bfloat16).contiguous(), x, bias, dx, part, dbias, accumulate=sink)
        if sink:
            grad_sink.done(pb)
            return dx, None
        return dx, dbias


def bias_gelu(x, bias):
    if not x.is_cuda:
        return torch.nn.functional.gelu(x.float() + bias)
    return _BiasGelu.apply(x.to(torch.bfloat16), bias)


# ---------------------------------------------------------------- attention softmax
class _AttnSoftmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, scores, mask, scale, p, rows_per_batch):
        C = _C()
        S = scores.contiguous()
        P = torch.empty_like(S)
        Pd = torch.empty_like(S) if p > 0 else None
        seed = next_seed() if p > 0 else 0
        C.softmax_fwd(S, mask, P, Pd, rows_per_batch, scale, p, seed)
        ctx.save_for_backward(P)
        ctx.scale, ctx.p, ctx.seed = scale, p, seed
        return Pd if Pd is not None else P

    @staticmethod
    def backward(ctx, dPd):
        C = _C()
        (P,) = ctx.saved_tensors
        dS = torch.empty_like(P)
        C.softmax_bwd(dPd.to(torch.bfloat16).contiguous(), P, dS, ctx.scale, ctx.p, ctx.seed)
        return dS, None, None, None, None


def attention_softmax(scores, mask: Optional[torch.Tensor], scale: float, p: float = 0.0, training: bool = True):
    """softmax(scale * scores + mask) with fused prob-dropout.

    scores [B, heads, Sq, Sk] (bf16 on GPU); mask [B, Sk] additive fp32 or None."""
    p = p if training else 0.0
    B, Hh, Sq, Sk = scores.shape
    if not scores.is_cuda:
        z = scores.float() * scale
        if mask is not None:
            z = z + mask.float()[:, None, None, :]
        pr = torch.softmax(z, -1)
        return torch.nn.functional.dropout(pr, p, True) if p > 0 else pr
    m = mask.float().contiguous() if mask is not None else None
    return _AttnSoftmax.apply(scores.to(torch.bfloat16), m, float(scale), float(p), Hh * Sq)


# ---------------------------------------------------------------- fused self-attention
class _FusedAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, bias, mask, nh, scale, p):
        C = _C()
        B, S, H3 = qkv.shape
        out = torch.empty(B, S, H3 // 3, dtype=torch.bfloat16, device=qkv.device)
        lse = torch.empty(B, nh, S, dtype=torch.float32, device=qkv.device)
        seed = next_seed() if p > 0 else 0
        C.attn_fwd(qkv, bias, mask, out, lse, nh, scale, p, seed)
        ctx.save_for_backward(qkv, bias if bias is not None else torch.empty(0, device=qkv.device),
                              mask if mask is not None else torch.empty(0, device=qkv.device), out, lse)
        ctx.has_bias, ctx.has_mask = bias is not None, mask is not None
        ctx.nh, ctx.scale, ctx.p, ctx.seed = nh, scale, p, seed
        ctx.bias_param = bias
        return out

    @staticmethod
    def backward(ctx, dout):
        C = _C()
        qkv, bias, mask, out, lse = ctx.saved_tensors
        dqkv = torch.empty_like(qkv)
        Dbuf = torch.empty_like(lse)
        dbias = bpart = None
        sink = False
        if ctx.has_bias and not _ATTN_BIAS_PARTIALS:   # A/B only: column sums re-read from dqkv
            C.attn_bwd(qkv, bias, mask if ctx.has_mask else None, out, dout.to(torch.bfloat16).contiguous(), lse,
                       Dbuf, dqkv, ctx.nh, ctx.scale, ctx.p, ctx.seed)
            H3 = dqkv.shape[-1]
            part = torch.empty(max(1, min(256, dqkv.numel() // H3 // 64)) * H3, dtype=torch.float32,
                               device=dqkv.device)
            pb = ctx.bias_param
            sink = grad_sink.all_enabled(pb)
            dbias = grad_sink.target(pb) if sink else torch.empty(H3, dtype=torch.float32, device=dqkv.device)
            C.colsum_bf16(dqkv.view(-1, H3), part, dbias, accumulate=sink)
            if sink:
                grad_sink.done(pb)
                dbias = None
            return dqkv, dbias, None, None, None, None
        if ctx.has_bias:
            # bias grad = column sums of dqkv: per-wave partials written by the
            # backward kernels themselves, reduced by one small pass (no re-read of dqkv)
            B, S, H3 = qkv.shape
            bpart = torch.empty(B * S // 16 * H3, dtype=torch.float32, device=qkv.device)
            pb = ctx.bias_param
            sink = grad_sink.all_enabled(pb)
            dbias = grad_sink.target(pb) if sink else torch.empty(H3, dtype=torch.float32, device=qkv.device)
        C.attn_bwd(qkv, bias if ctx.has_bias else None, mask if ctx.has_mask else None, out,
                   dout.to(torch.bfloat16).contiguous(), lse, Dbuf, dqkv, ctx.nh, ctx.scale, ctx.p, ctx.seed,
                   bpart, dbias, accumulate=sink)
        if sink:
            grad_sink.done(ctx.bias_param)
            dbias = None
        return dqkv, dbias, None, None, None, None


def attention_reference(qkv, bias, mask, nh: int, scale: float, p: float = 0.0):
    """softmax(scale * q k^T + mask) v per head from a packed [B, S, 3*H]
    projection (+ bias); fp32 PyTorch (CPU oracle / fallback)."""
    B, S, H3 = qkv.shape
    d = H3 // (3 * nh)
    x = qkv.float() + (bias.float() if bias is not None else 0.0)
    x = x.view(B, S, 3, nh, d)
    q, k, v = (x[:, :, i].permute(0, 2, 1, 3) for i in range(3))
    z = torch.matmul(q, k.transpose(-1, -2)) * scale
    if mask is not None:
        z = z + mask.float()[:, None, None, :]
    pr = torch.softmax(z, -1)
    if p > 0:
        pr = torch.nn.functional.dropout(pr, p, True)
    return torch.matmul(pr, v).permute(0, 2, 1, 3).reshape(B, S, nh * d)


def attention_supported(S: int, head_dim: int) -> bool:
    try:
        return bool(_C().attn_supported(S, head_dim))
    except Exception:   # extension not built: callers take the unfused path
        return False


def fused_attention(qkv, bias, mask: Optional[torch.Tensor], nh: int, scale: float, p: float = 0.0,
                    training: bool = True):
    """Multi-head self-attention straight from the packed QKV projection.

    qkv [B, S, 3*nh*64] (pre-bias GEMM output, bf16 on GPU), bias [3*nh*64]
    fp32 or None, mask [B, S] additive fp32 or None -> context [B, S, nh*64].
    GPU: csrc/kernels/attention.hip (one pass forward, two backward; prob
    dropout regenerated from its hash).  CPU: attention_reference."""
    p = p if training else 0.0
    if not qkv.is_cuda:
        return attention_reference(qkv, bias, mask, nh, scale, p)
    m = mask.float().contiguous() if mask is not None else None
    b = bias.float().contiguous() if bias is not None else None
    return _FusedAttention.apply(qkv.to(torch.bfloat16).contiguous(), b, m, int(nh), float(scale), float(p))


def gelu_ref(x):
    return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))
