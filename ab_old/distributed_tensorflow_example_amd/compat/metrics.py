"""Streaming metrics (tf.contrib.metrics.streaming_auc / streaming_accuracy).

Reference: `auc_op = tf.contrib.metrics.streaming_auc(sigmoid(py_x), y)`
evaluated batch after batch, local variables initialised by
local_variables_initializer (lr2.py:398-400,408,455-468).

streaming_auc keeps TF's four local variables -- `<name>/true_positives`,
`false_negatives`, `true_negatives`, `false_positives`, fp32 [num_thresholds]
-- at TF's thresholds (-1e-7, j/(T-1), 1+1e-7; predicted positive <=> p > t).
One update bins the batch over the T+1 intervals between thresholds with the
native `auc_hist` kernel (every threshold in one pass) and adds the suffix sums
to the four variables; the AUC is TF's compute_auc (trapezoid, epsilon 1e-6).
Returns (value, update_op): `value` reads the variables, `update_op` adds the
batch and evaluates to the post-update AUC, as in TF; fetched together in one
run, `value` is the pre-update AUC whatever the fetch order.
Across workers (sync_workers) the four variables are all-reduced when read.
"""
from __future__ import annotations

import torch

from .. import ops as _ops
from .graph import LOCAL_VARIABLES, Tensor, Variable


def streaming_auc(predictions, labels, weights=None, num_thresholds=200, metrics_collections=None,
                  updates_collections=None, curve="ROC", name=None, sync_workers=False):
    name = name or "auc"
    if num_thresholds < 2:
        raise ValueError("num_thresholds must be >= 2")
    if curve not in ("ROC", "PR"):
        raise ValueError("curve must be 'ROC' or 'PR'")

    def local(suffix):
        return Variable(torch.zeros(num_thresholds, dtype=torch.float32), trainable=False,
                        name=f"{name}/{suffix}", collections=[LOCAL_VARIABLES])

    tp, fn, tn, fp = (local(n) for n in ("true_positives", "false_negatives", "true_negatives", "false_positives"))
    cvars = (tp, fn, tn, fp)
    pre_key = f"auc-pre:{id(tp)}"

    def current():
        vals = [v.value.detach() for v in cvars]
        if sync_workers:
            from ..parallel.world import get_world

            w = get_world()
            if w.world_size > 1:
                vals = [x.clone() for x in vals]
                for x in vals:
                    w.all_reduce(x)
        return torch.tensor(_ops.auc_from_confusion(*vals, curve=curve))

    class _Value(Tensor):
        def _eval(self, ctx):
            return ctx.state[pre_key] if pre_key in ctx.state else current()

    class _Update(Tensor):
        def _eval(self, ctx):
            pred, lab = ctx.eval(predictions), ctx.eval(labels)
            wts = None if weights is None else ctx.eval(weights)
            ctx.state.setdefault(pre_key, current())       # a value fetched in the same run reads this
            with torch.no_grad():
                dev = pred.device if torch.is_tensor(pred) else torch.device("cpu")
                pos = torch.zeros(num_thresholds + 1, dtype=torch.int64 if wts is None else torch.float64, device=dev)
                neg = torch.zeros_like(pos)
                _ops.auc_histogram_(pred.detach().reshape(-1), lab.detach().reshape(-1), pos, neg, wts)
                for var, add in zip(cvars, _ops.auc_confusion(pos, neg)):
                    var.value.data += add.to(var.value.device)
            return current()

    # the graph edges stay explicit (the GraphDef export and the fused-step
    # lowering see that the AUC reads the predictions -- hence the weights a
    # train_op updates -- and the confusion variables); the custom _eval above
    # decides the values
    deps = [predictions, labels] + ([] if weights is None else [weights]) + list(cvars)
    val = _Value(None, list(cvars), name + "/value")
    upd = _Update(None, deps, name + "/update_op")
    from .graph import get_default_graph

    g = get_default_graph()
    for c in metrics_collections or ():
        g.add_to_collection(c, val)
    for c in updates_collections or ():
        g.add_to_collection(c, upd)
    return val, upd


def streaming_accuracy(predictions, labels, name="accuracy"):
    total = Variable(torch.zeros(1, dtype=torch.float64), trainable=False, name=name + "/total",
                     collections=[LOCAL_VARIABLES])
    count = Variable(torch.zeros(1, dtype=torch.float64), trainable=False, name=name + "/count",
                     collections=[LOCAL_VARIABLES])
    val = Tensor(lambda t, c: (t / c.clamp_min(1))[0], [total, count], name + "/value")

    def update(p, l, t, c):
        with torch.no_grad():
            t.data += (p.reshape(-1) == l.reshape(-1)).double().sum()
            c.data += p.numel()
        return (t / c.clamp_min(1))[0]
    return val, Tensor(update, [predictions, labels, total, count], name + "/update_op")


def accuracy(labels, predictions, name="accuracy"):
    return streaming_accuracy(predictions, labels, name)


def auc(labels, predictions, num_thresholds=200, name="auc"):
    return streaming_auc(predictions, labels, num_thresholds=num_thresholds, name=name)
