"""BERT-base masked-LM pretraining model (BASELINE config #4).

Not in the reference (SURVEY s2.7 lists it as a BASELINE extension); built on
the same runtime: fp32 master weights, bf16 activations, hipBLASLt for the
plain GEMMs and the framework's fused HIP kernels for everything around them:

  embeddings   word + position + type (fp32 sum) -> LN + dropout      (_EmbLN)
  attention    QKV one GEMM -> Q.K^T batched GEMM -> scale+mask+softmax
               +prob-dropout (one kernel) -> P.V -> out GEMM ->
               bias+dropout+residual+LN (one kernel)
  FFN          GEMM -> bias+GELU (one kernel) -> GEMM -> bias+dropout+residual+LN
  MLM head     only the masked positions (~15%): dense -> bias+GELU -> LN ->
               tied-decoder GEMM -> fused softmax-xent kernel

Data parallelism: parallel.ddp.DistributedDataParallel -- gradient-as-bucket
views, buckets launched on a comm stream as soon as backward fills them
(RCCL over xGMI overlapped with the remaining backward).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import os

import torch
import torch.nn.functional as F

from .. import ops
from ..ops import big_gemm
from ..ops import grad_sink
from ..ops import transformer as T


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    intermediate: int = 3072
    max_position: int = 512
    type_vocab: int = 2
    dropout: float = 0.1
    attn_dropout: float = 0.1
    ln_eps: float = 1e-12
    init_std: float = 0.02
    fused_attention: bool = True    # GPU: attention.hip straight from the packed QKV projection

    @staticmethod
    def base():
        return BertConfig()

    @staticmethod
    def tiny():
        return BertConfig(vocab_size=1024, hidden=256, layers=2, heads=4, intermediate=1024, max_position=128)


def _lin(o, i, std):
    return torch.nn.Parameter(torch.randn(o, i) * std)


class _ShadowLinear(torch.autograd.Function):
    """y = x @ w16^T with the optimizer-maintained bf16 shadow of the fp32
    master w (no per-step cast kernels); dW comes out of the bf16 GEMM in fp32
    directly (hipBLASLt out_dtype), straight into the DDP bucket."""

    @staticmethod
    def forward(ctx, x, w, w16, slot=None):
        ctx.save_for_backward(x, w16)
        ctx.w = w
        ctx.slot = slot
        x2 = x.reshape(-1, x.shape[-1])
        if big_gemm.use_native("fwd", x2.shape[0], w16.shape[0], x2.shape[1], x.device):
            return big_gemm.linear_fwd(x2, w16).view(*x.shape[:-1], w16.shape[0])
        return F.linear(x, w16)

    @staticmethod
    def backward(ctx, gy):
        x, w16 = ctx.saved_tensors
        gy = gy.to(w16.dtype)
        gy2, x2 = gy.reshape(-1, gy.shape[-1]), x.reshape(-1, x.shape[-1])
        extra = ctx.slot.take() if ctx.slot is not None else None
        native_dx = big_gemm.use_native("dx", gy2.shape[0], w16.shape[1], gy2.shape[1], gy.device)
        if extra is not None:   # residual-branch gradient of x folded in as the GEMM's beta = 1 term
            # in place: ds is a fresh buffer nobody else reads, and addmm_ on it
            # is one GEMM with beta = 1 (an out-of-place addmm would copy it first)
            e2 = extra.reshape(-1, x.shape[-1])
            gx = (big_gemm.linear_dx(gy2, w16, extra=e2) if native_dx else e2.addmm_(gy2, w16)).view(x.shape)
        else:
            gx = big_gemm.linear_dx(gy2, w16).view(x.shape) if native_dx else gy @ w16
        w = ctx.w
        if grad_sink.enabled(w) and (w.grad is None or w.grad.is_contiguous()):
            _wgrad(gy2, x2, into=grad_sink.target(w))
            grad_sink.done(w)
            return gx, None, None, None
        dw = _wgrad(gy2, x2)
        epoch = getattr(w, "_dtf_tied_epoch", None) if getattr(w, "_dtf_tied", False) else None
        if epoch is not None:
            # a tied weight (BERT's word embedding / MLM decoder) whose fused
            # embedding forward tagged it: that embedding's backward, which runs
            # after this one, scatters its rows into this same tensor instead of
            # a zeroed one that autograd would then add (ops/transformer.py _BertEmbed)
            w._dtf_tied_dw = (epoch, dw)
        return gx, dw, None, None


def _linear_dx(gy2, w16, extra=None):
    """dX = gy2 @ w16 on the engine use_native picks; `extra` (a residual
    branch's gradient of X) accumulated in place as the GEMM's beta = 1 term."""
    native = big_gemm.use_native("dx", gy2.shape[0], w16.shape[1], gy2.shape[1], gy2.device)
    if extra is not None:
        return big_gemm.linear_dx(gy2, w16, extra=extra) if native else extra.addmm_(gy2, w16)
    return big_gemm.linear_dx(gy2, w16) if native else gy2 @ w16


def _linear_dw(gy2, x2, w):
    """dW = gy2^T x2: sunk into the DDP bucket (returns None) or returned."""
    if grad_sink.enabled(w) and (w.grad is None or w.grad.is_contiguous()):
        _wgrad(gy2, x2, into=grad_sink.target(w))
        grad_sink.done(w)
        return None
    return _wgrad(gy2, x2)


class _FFN(torch.autograd.Function):
    """y = gelu(x W1^T + b1) W2^T: BERT's feed-forward block on the bf16 weight
    shadows, with GELU in the GEMM epilogues (gemm_big.hip gemm_8ph<EP>):
      forward   FFN-up writes the pre-activation u = x W1^T + b1 AND h = gelu(u)
                from one epilogue (gemm_gelu_aux), or hipBLASLt + bias_gelu_fwd;
      backward  dU = (gy W2) * gelu'(u) with the b1-gradient partial column sums
                in one epilogue (gemm_dgelu), or the dH GEMM + bias_gelu_bwd;
    each fused path only where the per-shape timing (ops.big_gemm use_gelu_aux /
    use_dgelu) beats the separate passes.  `slot`: LN2's residual gradient of x,
    accumulated by the dX GEMM (beta = 1)."""

    @staticmethod
    def forward(ctx, x, w1, w1_16, b1, w2, w2_16, slot):
        x2 = x.reshape(-1, x.shape[-1])
        M, F_, H = x2.shape[0], w1_16.shape[0], x2.shape[1]
        u = torch.empty(M, F_, device=x.device, dtype=x.dtype)
        h = torch.empty_like(u)
        ctx.biased = big_gemm.use_gelu_aux(M, F_, H, x.device) and T._C().gemm_gelu_aux(x2, False, w1_16, True,
                                                                                        h, u, b1)
        if not ctx.biased:      # u without b1; bias_gelu adds it
            if big_gemm.use_native("fwd", M, F_, H, x.device):
                big_gemm.linear_fwd(x2, w1_16, out=u)
            else:
                torch.mm(x2, w1_16.t(), out=u)
            T._C().bias_gelu_fwd(u, b1, h)
        ctx.save_for_backward(x2, u, h, w1_16, w2_16, b1)
        ctx.w1, ctx.b1, ctx.w2, ctx.slot, ctx.xshape = w1, b1, w2, slot, x.shape
        if big_gemm.use_native("fwd", M, w2_16.shape[0], F_, x.device):
            y = big_gemm.linear_fwd(h, w2_16)
        else:
            y = torch.mm(h, w2_16.t())
        return y.view(*x.shape[:-1], w2_16.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x2, u, h, w1_16, w2_16, b1 = ctx.saved_tensors
        gy2 = gy.to(w2_16.dtype).reshape(-1, gy.shape[-1])
        M, F_, K = u.shape[0], u.shape[1], gy2.shape[1]
        gw2 = _linear_dw(gy2, h, ctx.w2)
        C = T._C()
        pb = ctx.b1
        sink = grad_sink.all_enabled(pb)
        db = grad_sink.target(pb) if sink else torch.empty(F_, dtype=torch.float32, device=u.device)
        ub = None if ctx.biased else b1           # the bias still to add to the saved u
        du = torch.empty_like(u)
        fused = False
        if big_gemm.use_dgelu(M, F_, K, u.device):
            colpart = torch.empty((M // 128) * F_, dtype=torch.float32, device=u.device)
            fused = C.gemm_dgelu(gy2, False, w2_16, False, du, u, ub, colpart, db, accumulate=sink)
        if not fused:
            dh = _linear_dx(gy2, w2_16)
            part = torch.empty(big_gemm.gelu_bwd_slices(M) * F_, dtype=torch.float32, device=u.device)
            C.bias_gelu_bwd(dh, u, ub if ub is not None else torch.zeros_like(b1), du, part, db, accumulate=sink)
        if sink:
            grad_sink.done(pb)
            db = None
        extra = ctx.slot.take() if ctx.slot is not None else None
        gx = _linear_dx(du, w1_16, extra.reshape(-1, x2.shape[1]) if extra is not None else None)
        gw1 = _linear_dw(du, x2, ctx.w1)
        return gx.view(ctx.xshape), gw1, None, db, gw2, None, None


def _ffn(x, w1, b1, w2, slot=None):
    """gelu(x W1^T + b1) W2^T, fused on the bf16-shadow path."""
    w1_16, w2_16 = getattr(w1, "_shadow", None), getattr(w2, "_shadow", None)
    if w1_16 is not None and w2_16 is not None and x.is_cuda and x.dtype == w1_16.dtype:
        return _FFN.apply(x, w1, w1_16, b1, w2, w2_16, slot)
    return _mm(T.bias_gelu(_mm(x, w1, slot), b1), w2)


def _wgrad_split(T: int, out: int, inp: int) -> int:
    """Token-slab count for the weight-gradient GEMM.  dW = gy^T x has a long
    reduction (T = B*S tokens) and few output tiles (36-144 of 128x128 for
    BERT-base), so one hipBLASLt GEMM leaves most of the 256 CUs idle
    (~0.5 PFLOP/s measured, scripts/probes/wgrad_probe.py); slabs run as one batched
    GEMM with ~4 tile waves and are reduced in fp32 (1.5-2.5x faster)."""
    tiles = max(1, (out // 128) * (inp // 128))
    s = 1
    while s < 16 and tiles * s * 2 <= 1024 and T % (2 * s) == 0 and T // (2 * s) >= 512:
        s *= 2
    return s


def _wgrad(gy2, x2, into=None):
    """dW[out, in] = gy2[T, out]^T @ x2[T, in] in fp32 (accumulated into `into`)."""
    T, out = gy2.shape
    if gy2.is_cuda and big_gemm.use_native("dw", out, x2.shape[1], T, gy2.device):
        return big_gemm.linear_dw(gy2, x2, into=into)   # split-K over tokens: fp32 slabs + reduce into `into`
    return _wgrad_torch(gy2, x2, into)


def _wgrad_torch(gy2, x2, into=None):
    """_wgrad on hipBLASLt: token-slab batched GEMM + slab_sum."""
    T, out = gy2.shape
    s = _wgrad_split(T, out, x2.shape[1]) if gy2.is_cuda else 1
    if s == 1:
        if into is not None:
            return torch.addmm(into, gy2.t(), x2, out_dtype=torch.float32, out=into)
        return torch.mm(gy2.t(), x2, out_dtype=torch.float32)
    parts = torch.bmm(gy2.view(s, T // s, out).transpose(1, 2), x2.view(s, T // s, -1), out_dtype=torch.float32)
    from .. import _native
    if into is not None and into.is_contiguous():   # one pass: into += sum of the slabs
        _native.load().slab_sum(parts, into, accumulate=True)
        return into
    res = torch.empty(parts.shape[1:], dtype=torch.float32, device=parts.device)
    _native.load().slab_sum(parts, res, accumulate=False)
    if into is not None:
        return into.add_(res)
    return res


def _mm(x, w, slot=None):
    """x [.., in] @ w[out, in]^T in the activation dtype (bf16 on GPU).  `slot`
    (a GradSlot shared with the LN epilogue that also reads x) is only handed
    out when this GEMM takes the shadow path, whose backward consumes it."""
    w16 = getattr(w, "_shadow", None)
    if w16 is not None and x.is_cuda and x.dtype == w16.dtype:
        return _ShadowLinear.apply(x, w, w16, slot)
    return F.linear(x, w.to(x.dtype))


def _slot_for(x, w):
    w16 = getattr(w, "_shadow", None)
    return T.GradSlot() if (w16 is not None and x.is_cuda and x.dtype == w16.dtype) else None


def _lookup(table, ids):
    """Row gather whose backward is the framework's scatter-add kernel
    (torch's sort-based index backward is ~14% of a BERT step on MI355X)."""
    flat = ids.reshape(-1)
    if not table.is_cuda:
        return table[flat]
    offs = torch.arange(flat.numel() + 1, device=flat.device)
    return ops.embedding_bag(table, flat, offs, None, "sum")


class BertLayer(torch.nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        h, f, s = c.hidden, c.intermediate, c.init_std
        self.c = c
        self.w_qkv = _lin(3 * h, h, s)
        self.b_qkv = torch.nn.Parameter(torch.zeros(3 * h))
        self.w_o = _lin(h, h, s)
        self.b_o = torch.nn.Parameter(torch.zeros(h))
        self.ln1_g = torch.nn.Parameter(torch.ones(h))
        self.ln1_b = torch.nn.Parameter(torch.zeros(h))
        self.w_1 = _lin(f, h, s)
        self.b_1 = torch.nn.Parameter(torch.zeros(f))
        self.w_2 = _lin(h, f, s)
        self.b_2 = torch.nn.Parameter(torch.zeros(h))
        self.ln2_g = torch.nn.Parameter(torch.ones(h))
        self.ln2_b = torch.nn.Parameter(torch.zeros(h))

    def forward(self, x, mask):
        c = self.c
        B, S, H = x.shape
        nh, d = c.heads, H // c.heads
        slot_x = _slot_for(x, self.w_qkv)      # LN1's residual grad of x -> QKV GEMM's dX
        if x.is_cuda and c.fused_attention and T.attention_supported(S, d):
            # q/k/v read in place from the packed projection, bias fused (attention.hip)
            ctx = T.fused_attention(_mm(x, self.w_qkv, slot_x), self.b_qkv, mask, nh, 1.0 / math.sqrt(d),
                                    c.attn_dropout, self.training)
        else:
            qkv = (_mm(x, self.w_qkv, slot_x) + self.b_qkv.to(x.dtype)).view(B, S, 3, nh, d)
            q = qkv[:, :, 0].permute(0, 2, 1, 3)
            k = qkv[:, :, 1].permute(0, 2, 3, 1)
            v = qkv[:, :, 2].permute(0, 2, 1, 3)
            scores = torch.matmul(q, k)                                   # [B, nh, S, S]
            probs = T.attention_softmax(scores, mask, 1.0 / math.sqrt(d), c.attn_dropout, self.training)
            ctx = torch.matmul(probs.to(v.dtype), v).permute(0, 2, 1, 3).reshape(B, S, H)
        a = T.bias_dropout_residual_layernorm(_mm(ctx, self.w_o), self.b_o, x, self.ln1_g, self.ln1_b,
                                              c.dropout, c.ln_eps, self.training, residual_slot=slot_x)
        slot_a = _slot_for(a, self.w_1)        # LN2's residual grad of a -> W1 GEMM's dX
        pre = _ffn(a, self.w_1, self.b_1, self.w_2, slot_a)
        out = T.bias_dropout_residual_layernorm(pre, self.b_2, a, self.ln2_g, self.ln2_b,
                                                c.dropout, c.ln_eps, self.training, residual_slot=slot_a)
        return out


class BertForMLM(torch.nn.Module):
    def __init__(self, c: BertConfig = None, seed: int = 0):
        super().__init__()
        c = c or BertConfig.base()
        self.c = c
        g = torch.random.fork_rng(devices=[])
        with g:
            torch.manual_seed(seed)
            s = c.init_std
            self.word = torch.nn.Parameter(torch.randn(c.vocab_size, c.hidden) * s)
            self.pos = torch.nn.Parameter(torch.randn(c.max_position, c.hidden) * s)
            self.typ = torch.nn.Parameter(torch.randn(c.type_vocab, c.hidden) * s)
            self.emb_g = torch.nn.Parameter(torch.ones(c.hidden))
            self.emb_b = torch.nn.Parameter(torch.zeros(c.hidden))
            self.layers = torch.nn.ModuleList([BertLayer(c) for _ in range(c.layers)])
            self.head_w = _lin(c.hidden, c.hidden, s)
            self.head_b = torch.nn.Parameter(torch.zeros(c.hidden))
            self.head_g = torch.nn.Parameter(torch.ones(c.hidden))
            self.head_beta = torch.nn.Parameter(torch.zeros(c.hidden))
            self.dec_b = torch.nn.Parameter(torch.zeros(c.vocab_size))
        grad_sink.mark_tied(self.word)          # embedding lookup + MLM decoder

    def gemm_weights(self):
        ws = [self.head_w, self.word]
        for l in self.layers:
            ws += [l.w_qkv, l.w_o, l.w_1, l.w_2]
        return ws

    def attach_shadows(self, optimizer=None):
        """bf16 compute copies of every GEMM weight, refreshed by the fused
        optimizer kernel in the same pass that updates the fp32 master."""
        for w in self.gemm_weights():
            if not hasattr(w, "_shadow"):
                w._shadow = torch.empty_like(w, dtype=torch.bfloat16)
            if optimizer is not None:
                optimizer.attach_shadow(w, w._shadow)
            else:
                with torch.no_grad():
                    w._shadow.copy_(w)

    def forward(self, input_ids, token_type, attn_mask, mlm_positions, mlm_labels):
        """Returns the mean MLM loss over the masked positions.

        input_ids/token_type [B, S] int64; attn_mask [B, S] (1 keep, 0 pad);
        mlm_positions [M] flat indices into B*S; mlm_labels [M] int64."""
        c = self.c
        B, S = input_ids.shape
        if input_ids.is_cuda and c.type_vocab == 2 and os.environ.get("DTF_BERT_EMB_FUSED", "1") != "0":
            # gather + sum + LayerNorm + dropout in one kernel, its backward in three
            # (ops/transformer.py _BertEmbed)
            x = T.bert_embed(self.word, self.typ, self.pos, self.emb_g, self.emb_b, input_ids, token_type,
                             c.dropout, c.ln_eps, self.training)
        else:
            if c.type_vocab == 2:   # 2-row table: a lerp (reduction backward) beats contended scatter-adds
                typ = self.typ[0] + token_type.reshape(-1, 1).to(self.typ.dtype) * (self.typ[1] - self.typ[0])
            else:
                typ = _lookup(self.typ, token_type)
            emb = (_lookup(self.word, input_ids) + typ).view(B, S, c.hidden) + self.pos[:S].unsqueeze(0)
            x = T.layernorm_dropout(emb, self.emb_g, self.emb_b, c.dropout, c.ln_eps, self.training)
        act = torch.bfloat16 if x.is_cuda else torch.float32
        x = x.to(act)
        add_mask = (1.0 - attn_mask.float()) * -10000.0
        for layer in self.layers:
            x = layer(x, add_mask)
        h = x.reshape(B * S, c.hidden).index_select(0, mlm_positions)
        h = T.bias_gelu(_mm(h, self.head_w), self.head_b)
        zero = torch.zeros(c.hidden, device=h.device)
        h = T.bias_dropout_residual_layernorm(h, zero, None, self.head_g, self.head_beta, 0.0, c.ln_eps,
                                              self.training)
        return ops.softmax_xent(_mm(h, self.word), mlm_labels, bias=self.dec_b)   # bias fused in the xent kernels


def synthetic_mlm_batch(batch: int, seq: int, vocab: int, device, mask_prob: float = 0.15, seed: int = 0):
    """Random token ids with 15% MLM positions (fixed count per batch)."""
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, vocab, (batch, seq), generator=g)
    typ = torch.zeros(batch, seq, dtype=torch.int64)
    typ[:, seq // 2:] = 1
    am = torch.ones(batch, seq, dtype=torch.int64)
    m = max(1, int(round(batch * seq * mask_prob)))
    pos = torch.randperm(batch * seq, generator=g)[:m].sort().values
    labels = ids.reshape(-1)[pos].clone()
    ids.view(-1)[pos] = 103 % vocab                                  # [MASK]
    return tuple(t.to(device) for t in (ids, typ, am, pos, labels))
