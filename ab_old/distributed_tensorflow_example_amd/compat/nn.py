"""tf.nn subset used by the reference graphs, on the framework's fused ops."""
from __future__ import annotations

import torch

from .. import ops as _ops
from .graph import Tensor


def sigmoid(x, name="Sigmoid"):
    return Tensor(torch.sigmoid, [x], name, op_type="Sigmoid")


def relu(x, name="Relu"):
    return Tensor(torch.relu, [x], name, op_type="Relu")


def tanh(x, name="Tanh"):
    return Tensor(torch.tanh, [x], name, op_type="Tanh")


def gelu(x, name="Gelu"):
    return Tensor(torch.nn.functional.gelu, [x], name)


def softmax(logits, dim=-1, name="Softmax"):
    return Tensor(lambda t: torch.softmax(t, dim), [logits], name, op_type="Softmax", attrs={"dim": dim})


def log_softmax(logits, dim=-1, name="LogSoftmax"):
    return Tensor(lambda t: torch.log_softmax(t, dim), [logits], name, op_type="LogSoftmax", attrs={"dim": dim})


def bias_add(value, bias, name="BiasAdd"):
    return Tensor(lambda v, b: v + b, [value, bias], name, op_type="BiasAdd")


def xw_plus_b(x, w, b, name="xw_plus_b"):
    return Tensor(lambda a, ww, bb: _ops.linear_act(a, ww, bb, "none"), [x, w, b], name)


def dropout(x, keep_prob, seed=None, name="dropout"):
    return Tensor(lambda t, k: torch.nn.functional.dropout(t, 1.0 - float(k), True), [x, keep_prob], name)


def softmax_cross_entropy_with_logits(_sentinel=None, labels=None, logits=None, dim=-1, name=None):
    """per-row loss (TF returns a vector); reduce with reduce_mean."""
    def f(y, z):
        return -(y.float() * torch.log_softmax(z.float(), dim)).sum(dim)
    return Tensor(f, [labels, logits], name or "SoftmaxCrossEntropyWithLogits", op_type="SoftmaxCrossEntropyWithLogits",
                  attrs={"dim": dim})


def sparse_softmax_cross_entropy_with_logits(_sentinel=None, labels=None, logits=None, name=None):
    def f(y, z):
        return torch.nn.functional.cross_entropy(z.float(), y.long(), reduction="none")
    return Tensor(f, [labels, logits], name or "SparseSoftmaxCrossEntropyWithLogits",
                  op_type="SparseSoftmaxCrossEntropyWithLogits")


def sigmoid_cross_entropy_with_logits(*args, logits=None, labels=None, targets=None, name=None):
    """Accepts both the positional TF-0.12 form (logits, targets) used by
    lr2.py:391 and the keyword form (labels=, logits=)."""
    if args:
        logits = args[0] if logits is None else logits
        if len(args) > 1:
            targets = args[1]
    t = labels if labels is not None else targets
    return Tensor(lambda x, y: _ops.sigmoid_xent(x, y, reduction="none"), [logits, t],
                  name or "SigmoidCrossEntropyWithLogits")


def _partitioned(params):
    return getattr(params, "is_partitioned", False)


def embedding_lookup(params, ids, name="embedding_lookup"):
    if _partitioned(params):
        from .partitioned import lookup_dense

        t = Tensor(None, [ids], name)
        t._eval = lambda ctx: lookup_dense(ctx, params, ctx.eval(ids))
        return t
    return Tensor(lambda w, i: w[i.long()], [params, ids], name)


def embedding_lookup_sparse(params, sp_ids, sp_weights, combiner="mean", name="embedding_lookup_sparse"):
    """tf.nn.embedding_lookup_sparse on the fused embedding-bag kernel.

    sp_ids / sp_weights are SparseTensors over [batch, feature] (rows are bags);
    TF's default combiner is "mean", the reference passes combiner='sum'.
    """
    from .sparse import SparseTensor

    if _partitioned(params):
        from .partitioned import lookup_sparse

        t = Tensor(None, [sp_ids, sp_weights], name, op_type="EmbeddingLookupSparse", attrs={"combiner": combiner})
        t._eval = lambda ctx: lookup_sparse(ctx, params, ctx.eval(sp_ids),
                                            ctx.eval(sp_weights) if sp_weights is not None else None, combiner)
        t.params = params              # (compat/lowering.py matches lr2.py's graph through it)
        return t

    def f(w, ids_sp, wts_sp):
        offsets, ids, vals = SparseTensor.to_csr(ids_sp, wts_sp)
        out = _ops.embedding_bag(w, ids.to(w.device), offsets.to(w.device),
                                 None if vals is None else vals.to(w.device).float(), combiner)
        return out
    t = Tensor(f, [params, sp_ids, sp_weights], name, op_type="EmbeddingLookupSparse", attrs={"combiner": combiner})
    t.params = params
    return t


def l2_loss(t, name="L2Loss"):
    return Tensor(lambda x: (x.float() ** 2).sum() / 2, [t], name)


def in_top_k(predictions, targets, k, name="InTopK"):
    return Tensor(lambda p, t: (p.topk(k, 1).indices == t.long().unsqueeze(1)).any(1), [predictions, targets], name)
