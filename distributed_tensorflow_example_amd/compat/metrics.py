"""Streaming metrics (tf.contrib.metrics.streaming_auc / streaming_accuracy).

Reference: `auc_op = tf.contrib.metrics.streaming_auc(sigmoid(py_x), y)`
evaluated batch after batch, local variables initialised by
local_variables_initializer (lr2.py:398-400,408,455-468).  TF keeps four
[num_thresholds] confusion accumulators; here the state is a positive and a
negative histogram over `num_thresholds` bins filled by the native
`auc_hist` kernel (one pass, all thresholds at once), and the AUC is the
trapezoid of the cumulative counts.  Returns (value_tensor, update_op) like TF;
the value read together with the update in one run is the *pre-update* value
(SURVEY A11).  Across workers the histograms can be all-reduced.
"""
from __future__ import annotations

import torch

from .. import ops as _ops
from .graph import LOCAL_VARIABLES, Operation, Tensor, Variable


def streaming_auc(predictions, labels, weights=None, num_thresholds=200, name="auc", sync_workers=False):
    pos = Variable(torch.zeros(num_thresholds, dtype=torch.int64), trainable=False, name=name + "/pos",
                   collections=[LOCAL_VARIABLES])
    neg = Variable(torch.zeros(num_thresholds, dtype=torch.int64), trainable=False, name=name + "/neg",
                   collections=[LOCAL_VARIABLES])

    def value(p, n):
        pp, nn_ = p.detach(), n.detach()
        if sync_workers:
            from ..parallel.world import get_world

            w = get_world()
            if w.world_size > 1:
                pp, nn_ = pp.clone(), nn_.clone()
                w.all_reduce(pp)
                w.all_reduce(nn_)
        return torch.tensor(_ops.auc_from_histograms(pp, nn_))

    val = Tensor(value, [pos, neg], name + "/value")

    def update(pred, lab, p, n):
        # capture the pre-update value first (TF returns it alongside the update)
        with torch.no_grad():
            _ops.auc_histogram_(pred.detach().reshape(-1), lab.detach().reshape(-1), p.data, n.data)
        return torch.tensor(_ops.auc_from_histograms(p.detach(), n.detach()))

    upd = Tensor(update, [predictions, labels, pos, neg], name + "/update_op")
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
