"""Sparse logistic regression (lr2.py workload).

Reference model (lr2.py:368-400):
    W = Variable(random_normal([F, 1])), b = Variable(zeros([1]))
    py_x = embedding_lookup_sparse(W, sp_fids, sp_fvals, combiner='sum') + b
    loss = reduce_mean(sigmoid_cross_entropy_with_logits(py_x, y))
    GradientDescentOptimizer(lr).minimize(loss, global_step)
    auc = streaming_auc(sigmoid(py_x), y)

MI355X design: W is a row-sharded table (parallel.sharded_embedding, one
shard per GPU -- the ps role); b is replicated.  A step is: dedup + all-to-all
lookup, CSR bag kernel (sum of w*val), fused sigmoid-xent fwd/bwd kernel,
bag backward into [U,1], all-to-all of row gradients to their owners, fused
scatter-SGD apply.  Synchronous semantics: the loss is the mean over the
union of all workers' batches, so each owner applies lr/W times the sum of
the per-worker mean gradients (== lr x the global-batch gradient when the
per-worker batches are equal).
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from .. import ops
from ..parallel.sharded_embedding import ShardedEmbedding
from ..parallel.world import World, get_world


class SparseLRTrainer:
    def __init__(self, num_features: int, lr: float, world: Optional[World] = None, seed: int = 1,
                 init_std: float = 1.0, device=None, auc_bins: int = 200, ids_capacity: Optional[int] = None):
        self.world = world or get_world()
        self.device = torch.device(device) if device is not None else self.world.device
        self.lr = float(lr)
        self.W = ShardedEmbedding(num_features, 1, self.world, init_std=init_std, seed=seed, device=self.device,
                                  name="weights/Variable", capacity=ids_capacity)
        self.b = torch.zeros(1, dtype=torch.float32, device=self.device, requires_grad=True)
        self.global_step = 0
        self._graphed = None
        # streaming_auc's num_thresholds = auc_bins -> auc_bins + 1 histogram bins
        self.auc_pos = torch.zeros(auc_bins + 1, dtype=torch.int64, device=self.device)
        self.auc_neg = torch.zeros(auc_bins + 1, dtype=torch.int64, device=self.device)

    # ----------------------------------------------------------------- steps
    def _forward(self, batch):
        labels, offsets, ids, vals = batch.to(self.device) if hasattr(batch, "to") else batch
        out, st = self.W.bag_forward(ids, offsets, vals, "sum")
        return out + self.b, labels, st

    def train_step(self, batch) -> torch.Tensor:
        if self._graphed is not None:
            labels, offsets, ids, vals = batch.to(self.device) if hasattr(batch, "to") else batch
            loss = self._graphed(labels, offsets, ids, vals)
            self.global_step += 1
            return loss.detach()
        return self._train_step(batch)

    def enable_graph(self, on: bool = True):
        """Replay each step as one captured hipGraph (GPU; needs the static
        device-resident routing: one worker, or an ids capacity for W > 1)."""
        from ..utils.graphs import GraphedStep

        if not on:
            self._graphed = None
            return
        if self.device.type != "cuda" or (self.world.world_size > 1 and self.W.capacity is None):
            raise RuntimeError("graph capture needs a GPU and static routing (ids_capacity for W > 1)")

        def step(labels, offsets, ids, vals):
            gs = self.global_step
            loss = self._train_step((labels, offsets, ids, vals))
            self.global_step = gs          # counted by train_step, not by warmup/capture
            return loss
        self._graphed = GraphedStep(step, lambda: [self.W.local, self.b.data])

    def _train_step(self, batch) -> torch.Tensor:
        logits, labels, st = self._forward(batch)
        loss = ops.sigmoid_xent(logits, labels)
        if self.b.grad is not None:
            self.b.grad = None
        loss.backward()
        ws = self.world.world_size
        self.W.bag_backward_sgd(st, self.lr / ws)
        with torch.no_grad():
            gb = self.b.grad.clone()
            if ws > 1:
                self.world.all_reduce(gb)
            self.b -= (self.lr / ws) * gb
        self.global_step += 1
        return loss.detach()

    @torch.no_grad()
    def evaluate(self, batch):
        """(mean loss, probabilities) without updating (lr2.py Test(), :307-315)."""
        logits, labels, _ = self._forward(batch)
        return ops.sigmoid_xent(logits, labels).detach(), torch.sigmoid(logits).reshape(-1)

    @torch.no_grad()
    def auc_update(self, batch):
        logits, labels, _ = self._forward(batch)
        ops.auc_histogram_(torch.sigmoid(logits).reshape(-1), labels.reshape(-1), self.auc_pos, self.auc_neg)

    def auc(self, all_workers: bool = True) -> float:
        pos, neg = self.auc_pos.clone(), self.auc_neg.clone()
        if all_workers and self.world.world_size > 1:
            self.world.all_reduce(pos)
            self.world.all_reduce(neg)
        return ops.auc_from_histograms(pos, neg)

    def reset_auc(self):
        self.auc_pos.zero_()
        self.auc_neg.zero_()

    # ----------------------------------------------------------------- state
    def checkpoint_tensors(self):
        local = {"weights/Variable": self.W}      # saved as a TF partitioned variable
        repl = {"bias/Variable": self.b.detach(), "global_step": torch.tensor(float(self.global_step))}
        return local, repl


def reference_loss_grad(W: torch.Tensor, b: torch.Tensor, labels, offsets, ids, vals):
    """fp64 oracle: loss and dense gradients of the lr2.py graph."""
    W = W.double().detach().requires_grad_(True)
    b = b.double().detach().requires_grad_(True)
    seg = torch.repeat_interleave(torch.arange(len(offsets) - 1), torch.diff(offsets))
    z = torch.zeros(len(offsets) - 1, dtype=torch.float64).index_add(0, seg, W[ids, 0] * vals.double()) + b
    y = labels.double().reshape(-1)
    loss = torch.nn.functional.binary_cross_entropy_with_logits(z, y)
    loss.backward()
    return loss.detach(), W.grad, b.grad


def steps_per_epoch(world: World, local_batches: int) -> int:
    """Synchronous DP needs the same step count on every worker: min over ranks."""
    if world.world_size == 1:
        return local_batches
    return int(-world.host_all_reduce(-float(local_batches), "max"))


def np_sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))
