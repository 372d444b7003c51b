"""Framework ops: autograd functions over the hand-written CDNA4 HIP kernels.

GPU tensors always take the native path (csrc/kernels/*.hip); if the
extension is missing on a GPU box the op raises -- there is no silent eager
fallback.  CPU tensors use plain PyTorch (the CPU/gloo configuration and the
numerics oracle in tests).

Reference op map: linear_act = MatMul + Add + Sigmoid/Relu
(example.py:95-97), softmax_xent (example.py:98-103), sigmoid_xent
(lr2.py:391), embedding_bag (tf.nn.embedding_lookup_sparse, lr2.py:390),
accuracy (example.py:125-128), AUC histograms (streaming_auc, lr2.py:400).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _native

ACT = {"none": 0, None: 0, "linear": 0, "relu": 1, "sigmoid": 2, "tanh": 3, "gelu": 4}
EMB_MODE = {"sum": 0, "mean": 1, "sqrtn": 2}


def _C():
    return _native.load()


def _act_cpu(z, act):
    a = ACT[act]
    if a == 1:
        return torch.relu(z)
    if a == 2:
        return torch.sigmoid(z)
    if a == 3:
        return torch.tanh(z)
    if a == 4:
        return torch.nn.functional.gelu(z)
    return z


# --------------------------------------------------------------------------- GEMM
def matmul(a: torch.Tensor, b: torch.Tensor, trans_a: bool = False, trans_b: bool = False,
           bias=None, act="none", out_dtype=None) -> torch.Tensor:
    """act(op(a) @ op(b) + bias) on the MFMA GEMM (no autograd): fp32 operands on
    the exact-f32 MFMA kernel, bf16 / mixed operands on the bf16 one."""
    if not a.is_cuda:
        A = a.t() if trans_a else a
        Bm = b.t() if trans_b else b
        z = A.float() @ Bm.float()
        if bias is not None:
            z = z + bias
        return _act_cpu(z, act).to(out_dtype or torch.float32)
    a = a if a.stride(-1) == 1 else a.contiguous()
    b = b if b.stride(-1) == 1 else b.contiguous()
    M = a.shape[1] if trans_a else a.shape[0]
    N = b.shape[0] if trans_b else b.shape[1]
    out = torch.empty((M, N), dtype=out_dtype or torch.float32, device=a.device)
    _C().gemm(a, trans_a, b, trans_b, out, bias, ACT[act], 1.0, 0.0, None)
    return out


class _LinearAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act):
        C = _C()
        x2 = x.reshape(-1, x.shape[-1])
        x2 = x2 if x2.stride(-1) == 1 else x2.contiguous()
        M, N = x2.shape[0], w.shape[1]
        y = torch.empty((M, N), dtype=torch.float32, device=x.device)
        z = torch.empty_like(y) if ACT[act] == 4 else None
        C.gemm(x2, False, w.contiguous(), False, y, b.contiguous() if b is not None else None, ACT[act],
               1.0, 0.0, z)
        ctx.save_for_backward(x2, w, y if z is None else z)
        ctx.act = ACT[act]
        ctx.has_b = b is not None
        ctx.b = b
        ctx.xshape = x.shape
        return y.reshape(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, gy):
        C = _C()
        x2, w, yz = ctx.saved_tensors
        gy = gy.reshape(-1, w.shape[1]).contiguous().float()
        if ctx.act != 0:
            dz = torch.empty_like(gy)
            if ctx.act == 4:
                C.act_backward(gy, None, yz, dz, 4)
            else:
                C.act_backward(gy, yz, None, dz, ctx.act)
        else:
            dz = gy
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty((dz.shape[0], w.shape[0]), dtype=torch.float32, device=dz.device)
            C.gemm(dz, False, w.contiguous(), True, gx, None, 0, 1.0, 0.0, None)   # dZ W^T
            gx = gx.reshape(ctx.xshape)
        from . import grad_sink
        if ctx.needs_input_grad[1]:
            if grad_sink.all_enabled(w):
                # sunk: X^T dZ accumulated straight into w.grad (beta = 1: no zeroed
                # temporary, no AccumulateGrad add)
                C.gemm(x2, True, dz, False, grad_sink.target(w), None, 0, 1.0, 1.0, None)
                grad_sink.done(w)
            else:
                gw = torch.empty_like(w, dtype=torch.float32)
                C.gemm(x2, True, dz, False, gw, None, 0, 1.0, 0.0, None)                # X^T dZ
        if ctx.has_b and ctx.needs_input_grad[2]:
            b = ctx.b
            if grad_sink.all_enabled(b):
                C.col_sum(dz, grad_sink.target(b), True)
                grad_sink.done(b)
            else:
                gb = torch.empty(w.shape[1], dtype=torch.float32, device=dz.device)
                C.col_sum(dz, gb)
        return gx, gw, gb, None


def linear_act(x: torch.Tensor, w: torch.Tensor, b=None, act="none") -> torch.Tensor:
    """y = act(x @ w + b), w: [in, out] (TF layout), fused bias + activation epilogue."""
    if not x.is_cuda:
        z = x.float() @ w
        if b is not None:
            z = z + b
        return _act_cpu(z, act)
    return _LinearAct.apply(x, w, b, act)


class Linear(torch.nn.Module):
    """Dense layer with TF-layout weight [in, out] on the fused MFMA GEMM."""

    def __init__(self, fan_in, fan_out, act="none", bias=True, init_std=None):
        super().__init__()
        std = init_std if init_std is not None else (1.0 / fan_in) ** 0.5
        self.weight = torch.nn.Parameter(torch.randn(fan_in, fan_out) * std)
        self.bias = torch.nn.Parameter(torch.zeros(fan_out)) if bias else None
        self.act = act

    def forward(self, x):
        return linear_act(x, self.weight, self.bias, self.act)


# --------------------------------------------------------------------------- losses
class _SoftmaxXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, dense, naive):
        C = _C()
        lg = logits.contiguous().float()
        Bn = lg.shape[0]
        loss_rows = torch.empty(Bn, dtype=torch.float32, device=lg.device)
        grad = torch.empty_like(lg)
        if dense:
            C.softmax_xent(lg, None, labels.contiguous().float(), loss_rows, grad, None, 1.0 / Bn, naive)
        else:
            C.softmax_xent(lg, labels.contiguous().long(), None, loss_rows, grad, None, 1.0 / Bn, naive)
        ctx.save_for_backward(grad)
        return loss_rows.mean()

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        return grad * g, None, None, None


class _XentBF16(torch.autograd.Function):
    """Vocab-sized rows: bf16 logits (+ fp32 bias) read once forward, once backward."""

    @staticmethod
    def forward(ctx, logits, bias, labels):
        C = _C()
        Bn = logits.shape[0]
        lse = torch.empty(Bn, dtype=torch.float32, device=logits.device)
        loss_rows = torch.empty_like(lse)
        C.xent_fwd_bf16(logits, bias, labels, lse, loss_rows)
        ctx.save_for_backward(logits, bias if bias is not None else torch.empty(0, device=logits.device), labels, lse)
        ctx.has_bias = bias is not None
        ctx.bias_param = bias
        return loss_rows.mean()

    @staticmethod
    def backward(ctx, g):
        C = _C()
        logits, bias, labels, lse = ctx.saved_tensors
        grad = torch.empty_like(logits)
        C.xent_bwd_bf16(logits, bias if ctx.has_bias else None, labels, lse, g.float().reshape(1).contiguous(), grad,
                        1.0 / logits.shape[0])
        dbias = None
        if ctx.has_bias:
            from . import grad_sink
            # column sums on the in-tree two-stage kernel (torch's bf16 sum over the
            # [M, vocab] gradient was ~90 us of a BERT-base step); sunk into
            # .grad when the bias carries a DDP sink
            V = grad.shape[-1]
            rows = grad.numel() // V
            if V % 2 or grad.data_ptr() % 4:
                return grad, grad.sum(0, dtype=torch.float32).reshape(bias.shape), None
            part = torch.empty(max(1, min(256, rows // 64)) * V, dtype=torch.float32, device=grad.device)
            pb = ctx.bias_param
            sink = pb is not None and grad_sink.all_enabled(pb)
            out = grad_sink.target(pb) if sink else torch.empty(V, dtype=torch.float32, device=grad.device)
            C.colsum_bf16(grad.reshape(rows, V), part, out, accumulate=sink)
            if sink:
                grad_sink.done(pb)
            else:
                dbias = out.reshape(bias.shape)
        return grad, dbias, None


def softmax_xent(logits, labels, naive: bool = False, bias=None):
    """mean softmax cross-entropy; labels: int class ids [B] or dense [B, C].

    `bias` [C] (optional) is added to the logits inside the kernels; bf16 GPU
    logits with int labels take the vocab-row kernels (no fp32 copy)."""
    dense = labels.dim() == 2
    if (logits.is_cuda and logits.dtype == torch.bfloat16 and not dense and not naive
            and logits.dim() == 2 and logits.shape[1] % 2 == 0):
        b = bias.float().contiguous() if bias is not None else None
        return _XentBF16.apply(logits.contiguous(), b, labels.contiguous().long())
    if bias is not None:
        logits = logits.float() + bias.float()
    if not logits.is_cuda:
        logp = torch.log_softmax(logits.float(), 1)
        if naive:
            logp = torch.log(torch.softmax(logits.float(), 1))
        if dense:
            return (-(labels.float() * logp).sum(1)).mean()
        return torch.nn.functional.nll_loss(logp, labels.long())
    return _SoftmaxXent.apply(logits, labels, dense, naive)


class _SigmoidXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, t, reduction):
        C = _C()
        xf = x.contiguous().float()
        tf_ = t.contiguous().float().reshape(xf.shape)
        loss = torch.empty_like(xf)
        n = xf.numel()
        grad = torch.empty_like(xf)
        C.sigmoid_xent(xf, tf_, loss, grad, 1.0 / n if reduction == "mean" else 1.0)
        ctx.save_for_backward(grad)
        ctx.reduction = reduction
        return loss.mean() if reduction == "mean" else (loss.sum() if reduction == "sum" else loss)

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        return grad * g, None, None


class _Logit3Xent(torch.autograd.Function):
    """mean sigmoid-xent(a + b + bias, t) in one kernel, backward in one more
    (the bias gradient stored, or sunk into bias.grad: ops/grad_sink.py)."""

    @staticmethod
    def forward(ctx, a, b, bias, t):
        C = _C()
        af, bf = a.contiguous().float().reshape(-1), b.contiguous().float().reshape(-1)
        loss = torch.empty(1, dtype=torch.float32, device=a.device)
        dz = torch.empty_like(af)
        C.logit3_xent(af, bf, bias.contiguous().float().reshape(-1), t.contiguous().float().reshape(-1), loss, dz)
        ctx.save_for_backward(dz)
        ctx.bias = bias
        ctx.shapes = (a.shape, b.shape)
        return loss.reshape(())

    @staticmethod
    def backward(ctx, g):
        from . import grad_sink
        (dz,) = ctx.saved_tensors
        d = torch.empty_like(dz)
        bias = ctx.bias
        sink = ctx.needs_input_grad[2] and grad_sink.all_enabled(bias)
        gb = None
        if sink:
            _C().logit3_xent_bwd(dz, g.contiguous().float().reshape(1), d, grad_sink.target(bias), True)
            grad_sink.done(bias)
        else:
            gb = torch.empty(1, dtype=torch.float32, device=dz.device) if ctx.needs_input_grad[2] else None
            _C().logit3_xent_bwd(dz, g.contiguous().float().reshape(1), d, gb, False)
            gb = None if gb is None else gb.reshape(bias.shape)
        return d.view(ctx.shapes[0]), d.view(ctx.shapes[1]), gb, None


def logit3_xent(a, b, bias, targets):
    """mean(sigmoid_cross_entropy_with_logits(a + b + bias, targets)) -- the
    Wide&Deep head (wide part + tower output + shared bias) fused."""
    if not a.is_cuda:
        return sigmoid_xent(a + b + bias, targets)
    return _Logit3Xent.apply(a, b, bias, targets)


def multi_copy_(dsts, srcs):
    """dst.copy_(src) for every pair, one kernel on the GPU (contiguous pairs of
    one dtype / size, at most 8); elementwise copies otherwise."""
    if (dsts and all(d.is_cuda and s.is_cuda and d.is_contiguous() and s.is_contiguous() and d.dtype == s.dtype
                     and d.numel() == s.numel() for d, s in zip(dsts, srcs)) and len(dsts) <= 8):
        _C().multi_copy(list(dsts), list(srcs))
        return
    for d, s in zip(dsts, srcs):
        d.copy_(s, non_blocking=True)


def sigmoid_xent(logits, targets, reduction: str = "mean"):
    """tf.nn.sigmoid_cross_entropy_with_logits (+ reduction), fused fwd/bwd."""
    if not logits.is_cuda:
        loss = torch.nn.functional.binary_cross_entropy_with_logits(
            logits.float(), targets.float().reshape(logits.shape), reduction=reduction)
        return loss
    if reduction not in ("mean", "sum"):
        x = logits.float()
        t = targets.float().reshape(x.shape)
        return torch.clamp(x, min=0) - x * t + torch.log1p(torch.exp(-x.abs()))
    return _SigmoidXent.apply(logits, targets, reduction)


# --------------------------------------------------------------------------- embeddings
class _EmbeddingBag(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weight, ids, offsets, psw, mode, table=None, remap=None):
        """table / remap (one-GPU sharded tables): the rows are read in place as
        table[remap[ids]]; `weight` is then only the [U, D] gradient target
        (never read -- an uninitialised tensor is fine)."""
        C = _C()
        B = offsets.numel() - 1
        D = 1 if weight.dim() == 1 else weight.shape[1]
        out = torch.empty((B, D), dtype=torch.float32, device=weight.device)
        if table is not None:
            C.embedding_bag_fwd(table, ids, offsets, psw, EMB_MODE[mode], out, None, remap)
        else:
            C.embedding_bag_fwd(weight.contiguous(), ids, offsets, psw, EMB_MODE[mode], out, None)
        ctx.save_for_backward(ids, offsets, psw if psw is not None else torch.empty(0))
        ctx.has_psw = psw is not None
        ctx.mode = mode
        ctx.wshape = weight.shape
        return out

    @staticmethod
    def backward(ctx, gout):
        C = _C()
        ids, offsets, psw = ctx.saved_tensors
        gw = torch.zeros(ctx.wshape, dtype=torch.float32, device=gout.device)
        psw = psw if ctx.has_psw else None
        if ctx.mode == "sum" and 0 < ids.numel() < 2 ** 31 and ctx.wshape[0] < 2 ** 31:
            rows, occ, bag_of = _bag_plan(ids, offsets)
            C.embedding_bag_bwd_sorted(gw, rows, occ, bag_of, psw, gout.reshape(offsets.numel() - 1, -1)
                                       .contiguous().float())
        else:
            C.embedding_bag_bwd(gw, ids, offsets, psw, gout.contiguous().float(), EMB_MODE[ctx.mode], 0.0)
        return gw, None, None, None, None, None, None


_SORT_PLAN = [None]   # (key, ids ref, (rows int32 sorted, occ))
_BAG_OF = [None]      # (key, offsets ref, bag_of int32)
# bumped around every hipGraph capture (utils/graphs.py): a plan computed
# eagerly (e.g. by the capture's warmup on the same static input buffers) must
# never be baked into a graph -- it would freeze the warmup batch's bag map
_CAPTURE_EPOCH = [0]


def bump_capture_epoch() -> None:
    _CAPTURE_EPOCH[0] += 1


def _tkey(t: torch.Tensor):
    return (t.data_ptr(), t.numel(), t._version, _CAPTURE_EPOCH[0])


def register_sorted_ids(ids: torch.Tensor, rows_sorted: torch.Tensor, occ: torch.Tensor) -> None:
    """Hand the bag backward a sort of `ids` that the caller already has (the
    sharded-table router sorts ids to dedup them; the dedup inverse it produces
    is monotone in the ids, so the same permutation sorts the inverse)."""
    _SORT_PLAN[0] = (_tkey(ids), ids, (rows_sorted.to(torch.int32).contiguous(), occ.contiguous()))


def _bag_plan(ids: torch.Tensor, offsets: torch.Tensor):
    """(rows int32 sorted, CSR position of each sorted occurrence, bag of each
    CSR position) for the sorted-segment bag backward.  The last sort and bag
    map are kept (with strong refs, so their data pointers cannot be recycled):
    the wide and deep tables of one Wide&Deep step read the same ids and share
    one sort, which the router usually supplied already."""
    c = _SORT_PLAN[0]
    if c is None or c[0] != _tkey(ids):
        rows, occ = torch.sort(ids.to(torch.int32))
        c = (_tkey(ids), ids, (rows.contiguous(), occ.contiguous()))
        _SORT_PLAN[0] = c
    b = _BAG_OF[0]
    if b is None or b[0] != _tkey(offsets):
        bag_of = torch.empty(ids.numel(), dtype=torch.int32, device=ids.device)
        _C().bag_index(offsets.long().contiguous(), bag_of)       # one kernel (repeat_interleave: five)
        b = (_tkey(offsets), offsets, bag_of)
        _BAG_OF[0] = b
    return c[2][0], c[2][1], b[2]


def embedding_bag(weight, ids, offsets, per_sample_weights=None, mode: str = "sum", table=None, remap=None):
    """Bag-combine rows of `weight` [V, D] for CSR bags (offsets [B+1]).

    == tf.nn.embedding_lookup_sparse(W, sp_ids, sp_weights, combiner=mode).
    table / remap (GPU): read row table[remap[id]] in place of weight[id] --
    `weight` ([len(remap), D]) is then only where the gradient goes.
    """
    ids = ids.long()
    offsets = offsets.long()
    if table is not None and not weight.is_cuda:
        weight = table.index_select(0, remap.clamp_min(0)).requires_grad_(weight.requires_grad)
        table = remap = None
    if not weight.is_cuda:
        W = weight if weight.dim() == 2 else weight.reshape(-1, 1)
        out = torch.nn.functional.embedding_bag(ids, W, offsets[:-1], mode="sum",
                                                per_sample_weights=per_sample_weights,
                                                include_last_offset=False)
        if mode != "sum":
            w = per_sample_weights if per_sample_weights is not None else torch.ones_like(ids, dtype=W.dtype)
            seg = torch.repeat_interleave(torch.arange(offsets.numel() - 1), offsets[1:] - offsets[:-1])
            den = torch.zeros(offsets.numel() - 1, dtype=W.dtype).index_add_(0, seg, w if mode == "mean" else w * w)
            den = den if mode == "mean" else den.sqrt()
            out = out / den.clamp_min(1e-30).unsqueeze(1)
        return out
    psw = per_sample_weights.contiguous().float() if per_sample_weights is not None else None
    if table is not None:
        t = table if table.dim() == 2 else table.reshape(-1, 1)
        return _EmbeddingBag.apply(weight, ids.contiguous(), offsets.contiguous(), psw, mode, t.contiguous(),
                                   remap.long().contiguous())
    return _EmbeddingBag.apply(weight, ids.contiguous(), offsets.contiguous(), psw, mode)


def embedding_bag_sgd_(weight, ids, offsets, per_sample_weights, grad_out, lr: float, mode: str = "sum"):
    """Fused sparse SGD: weight[ids] -= lr * w * grad_out[bag]  (ScatterSub apply).
    offsets None: one id per bag (row i of grad_out goes to weight[ids[i]])."""
    if not weight.is_cuda:
        if offsets is None:
            offsets = torch.arange(ids.numel() + 1, device=ids.device)
        seg = torch.repeat_interleave(torch.arange(offsets.numel() - 1), offsets[1:] - offsets[:-1])
        w = per_sample_weights if per_sample_weights is not None else torch.ones(ids.numel())
        W = weight if weight.dim() == 2 else weight.view(-1, 1)
        ok = (ids >= 0) & (ids < W.shape[0])               # -1 = routing padding (skipped, as on the GPU)
        W.index_add_(0, ids.long().clamp(0, max(W.shape[0] - 1, 0)),
                     -lr * (w * ok).unsqueeze(1) * grad_out[seg])
        return weight
    _C().embedding_bag_bwd(weight, ids.long().contiguous(), None if offsets is None else offsets.long().contiguous(),
                           per_sample_weights.contiguous().float() if per_sample_weights is not None else None,
                           grad_out.contiguous().float(), EMB_MODE[mode], float(lr))
    return weight


# --------------------------------------------------------------------------- metrics
def argmax_correct(logits, labels) -> torch.Tensor:
    """number of rows whose argmax equals the label (int64 tensor, on device)."""
    if not logits.is_cuda:
        return (logits.argmax(1) == labels.long()).sum()
    cnt = torch.zeros(1, dtype=torch.int64, device=logits.device)
    _C().argmax_correct(logits.contiguous().float(), labels.long().contiguous(), cnt)
    return cnt[0]


def auc_thresholds(num_thresholds: int) -> torch.Tensor:
    """streaming_auc's fp32 thresholds: -1e-7, j/(T-1) for 0 < j < T-1, 1 + 1e-7 (TF contrib.metrics)."""
    t = [0.0 - 1e-7] + [(i + 1) * 1.0 / (num_thresholds - 1) for i in range(num_thresholds - 2)] + [1.0 + 1e-7]
    return torch.tensor(t, dtype=torch.float32)


def auc_histogram_(pred, labels, pos_counts, neg_counts, weights=None):
    """Accumulate positive / negative histograms of predictions over the T + 1
    bins between streaming_auc's T thresholds (len(pos_counts) = T + 1): bin k
    holds predictions p with #{i : t_i < p} = k.  Labels: nonzero = positive."""
    nb = pos_counts.numel()
    if nb < 3:
        raise ValueError("need num_thresholds >= 2 (T + 1 >= 3 bins)")
    if not pred.is_cuda or weights is not None:
        p = pred.detach().float().reshape(-1).cpu()
        b = torch.searchsorted(auc_thresholds(nb - 1), p.contiguous())
        lab = labels.detach().reshape(-1).cpu() != 0
        wt = None if weights is None else torch.broadcast_to(torch.as_tensor(weights).float().cpu(), p.shape).reshape(-1)
        pos_counts += torch.bincount(b[lab], weights=None if wt is None else wt[lab], minlength=nb).to(
            pos_counts.device, pos_counts.dtype)
        neg_counts += torch.bincount(b[~lab], weights=None if wt is None else wt[~lab], minlength=nb).to(
            neg_counts.device, neg_counts.dtype)
        return
    _C().auc_hist(pred.contiguous().float().reshape(-1), labels.contiguous().float().reshape(-1),
                  pos_counts, neg_counts)


def auc_confusion(pos, neg):
    """(tp, fn, tn, fp) per threshold, fp32 like TF's local variables, from T+1-bin histograms."""
    pos = pos.detach().double().cpu()
    neg = neg.detach().double().cpu()
    tp = pos.flip(0).cumsum(0).flip(0)[1:]          # sum over bins k > i
    fp = neg.flip(0).cumsum(0).flip(0)[1:]
    return (tp.float(), (pos.sum() - tp).float(), (neg.sum() - fp).float(), fp.float())


def auc_from_confusion(tp, fn, tn, fp, curve: str = "ROC") -> float:
    """TF contrib.metrics compute_auc: trapezoid over thresholds, epsilon 1e-6, fp32."""
    eps = 1e-6
    tp, fn, tn, fp = (torch.as_tensor(v).float().cpu() for v in (tp, fn, tn, fp))
    rec = (tp + eps) / (tp + fn + eps)
    if curve == "ROC":
        x = fp / (fp + tn + eps)
        y = rec
    else:
        x = rec
        y = (tp + eps) / (tp + fp + eps)
    return float(torch.sum((x[:-1] - x[1:]) * (y[:-1] + y[1:]) / 2.0))


def auc_from_histograms(pos, neg, curve: str = "ROC") -> float:
    """streaming_auc's value from T+1-bin positive / negative histograms."""
    return auc_from_confusion(*auc_confusion(pos, neg), curve=curve)


# --------------------------------------------------------------------------- random init
_PHILOX_M0, _PHILOX_M1 = 0xD2511F53, 0xCD9E8D57
_PHILOX_W0, _PHILOX_W1 = 0x9E3779B9, 0xBB67AE85
_U32 = 0xFFFFFFFF


def philox4x32_10(c0, c1, c2, c3, k0: int, k1: int):
    """Philox4x32-10 (Salmon et al., SC'11) on uint64 arrays holding 32-bit words."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) for c in (c0, c1, c2, c3))
    m0, m1, sh, mask = np.uint64(_PHILOX_M0), np.uint64(_PHILOX_M1), np.uint64(32), np.uint64(_U32)
    for _ in range(10):
        p0 = m0 * c0
        p1 = m1 * c2
        c0, c1, c2, c3 = (p1 >> sh) ^ c1 ^ np.uint64(k0), p1 & mask, (p0 >> sh) ^ c3 ^ np.uint64(k1), p0 & mask
        k0 = (k0 + _PHILOX_W0) & _U32
        k1 = (k1 + _PHILOX_W1) & _U32
    return c0, c1, c2, c3


def _philox10_np(q: np.ndarray, seed: int):
    """Counters (q_lo, q_hi, 0, 0) under key (seed_lo, seed_hi)."""
    z = np.zeros_like(q)
    return philox4x32_10(q & np.uint64(_U32), q >> np.uint64(32), z, z, seed & _U32, (seed >> 32) & _U32)


def _unit_np(x: np.ndarray) -> np.ndarray:
    return (((x & np.uint64(0x7FFFFF)) | np.uint64(0x3F800000)).astype(np.uint32).view(np.float32)
            - np.float32(1.0))


def philox_normal_(out: torch.Tensor, row_mul: int, row_add: int, seed: int, mean: float = 0.0,
                   stddev: float = 1.0, chunk_rows: int = 1 << 20) -> torch.Tensor:
    """out[r, c] = N(mean, stddev) of global element (r * row_mul + row_add) * dim + c.

    Counter-based (Philox4x32-10 + TF's Box-Muller), so a table row gets the
    same value on whichever rank holds it.  GPU: csrc/kernels/random.hip;
    CPU: the same algorithm in numpy (fp32 transcendentals; equal to a few ulp)."""
    assert out.dim() == 2 and out.dtype == torch.float32 and out.is_contiguous()
    seed = int(seed) & ((1 << 64) - 1)
    if out.is_cuda:
        _C().philox_normal(out, int(row_mul), int(row_add), seed, float(mean), float(stddev))
        return out
    rows, dim = out.shape
    for s in range(0, rows, chunk_rows):
        e = min(rows, s + chunk_rows)
        r = np.arange(s, e, dtype=np.uint64) * np.uint64(row_mul) + np.uint64(row_add)
        g = (r[:, None] * np.uint64(dim) + np.arange(dim, dtype=np.uint64)[None, :]).reshape(-1)
        c0, c1, c2, c3 = _philox10_np(g >> np.uint64(2), seed)
        w = (g & np.uint64(3)).astype(np.int64)
        x0 = np.where(w < 2, c0, c2)
        x1 = np.where(w < 2, c1, c3)
        u1 = np.maximum(_unit_np(x0), np.float32(1e-7))
        v1 = np.float32(6.2831853071795864769) * _unit_np(x1)
        rr = np.sqrt(np.float32(-2.0) * np.log(u1))
        z = np.where(w & 1, np.cos(v1) * rr, np.sin(v1) * rr).astype(np.float32)
        out[s:e] = torch.from_numpy((np.float32(mean) + np.float32(stddev) * z).reshape(e - s, dim))
    return out
