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
from ..parallel.sharded_embedding import ShardedEmbedding, StaticStepMixin, lookup_shared, pad_to_capacity
from ..parallel.world import World, get_world


class SparseLRTrainer(StaticStepMixin):
    def __init__(self, num_features: int, lr: float, world: Optional[World] = None, seed: int = 1,
                 init_std: float = 1.0, device=None, auc_bins: int = 200, ids_capacity: Optional[int] = None,
                 rows: int = 500, peer_capacity: Optional[int] = None, update_mode: Optional[str] = None,
                 use_locking: bool = False, table: Optional[ShardedEmbedding] = None,
                 bias: Optional[torch.Tensor] = None):
        """`table` / `bias`: train existing storage in place instead of creating
        it (the compat Session's lowered lr2 graph: a PartitionedVariable's
        shards and the `bias/Variable` tensor, compat/lowering.py)."""
        self.world = world or get_world()
        self.device = torch.device(device) if device is not None else self.world.device
        self.lr = float(lr)
        if table is not None:
            if table.dim != 1 or table.num_rows != num_features:
                raise ValueError("table must be [num_features, 1]")
            self.W = table
        else:
            self.W = ShardedEmbedding(num_features, 1, self.world, init_std=init_std, seed=seed, device=self.device,
                                      name="weights/Variable", capacity=ids_capacity, peer_capacity=peer_capacity)
        self.rows = int(rows)              # batch rows of the captured step (lr2: batch_size)
        self._window = []                  # static steps since the router's last check (replay source)
        self._example = None
        if bias is not None:
            if bias.numel() != 1 or bias.dtype != torch.float32:
                raise ValueError("bias must be one fp32 value")
            self.b = bias if bias.requires_grad else bias.requires_grad_(True)
        else:
            self.b = torch.zeros(1, dtype=torch.float32, device=self.device, requires_grad=True)
        self.global_step = 0
        self._graphed = None
        # streaming_auc's num_thresholds = auc_bins -> auc_bins + 1 histogram bins
        self.auc_pos = torch.zeros(auc_bins + 1, dtype=torch.int64, device=self.device)
        self.auc_neg = torch.zeros(auc_bins + 1, dtype=torch.int64, device=self.device)
        # 'async': the reference's rule (lr2.py:359-396, plain GradientDescentOptimizer
        # under replica_device_setter): every worker reads W's rows from -- and
        # scatters its update into -- the owners' shared shards, b lives in a shared
        # Hogwild store, global_step counts every worker's update; no collective
        from ..parallel import async_ps
        self.update_mode = async_ps.update_mode(update_mode)
        self._bstore = None
        if self.update_mode == "async" and self.world.world_size > 1:
            self.W.hogwild = async_ps.HogwildTable(self.W, self.world, use_locking=use_locking)
            self._bstore = async_ps.HogwildStore([self.b.data], self.world, use_locking=use_locking)

    # ----------------------------------------------------------------- steps
    def _forward(self, batch, exact: bool = False):
        labels, offsets, ids, vals = batch.to(self.device) if hasattr(batch, "to") else batch
        if self.W.hogwild is not None:      # asynchronous: the owners' shared shards, no collective
            rows, ctx = self.W.lookup(ids)
        else:
            ctx = self.W.route(ids, exact=exact)
            rows = lookup_shared([self.W], ctx)[0]
        rows = rows.detach().requires_grad_(True)
        out = ops.embedding_bag(rows, ctx.inverse, offsets.to(self.device).long(),
                                None if vals is None else vals.to(self.device).float(), "sum")
        return out + self.b, labels, (rows, ctx)

    def _static_batch(self, batch):
        labels, offsets, ids, vals = batch.to(self.device) if hasattr(batch, "to") else batch
        offsets = offsets.to(self.device).long()
        ids = ids.to(self.device)
        vals = None if vals is None else vals.to(self.device).float()
        self._last_empty = ids.numel() == 0
        if self.W.capacity is not None:      # fixed shapes for the captured / static step
            offsets, ids, vals = pad_to_capacity(offsets, ids, vals, self.W.capacity)
        return labels.to(self.device), offsets, ids, vals

    def _router(self):
        return self.W.router

    def _route_table(self):
        return self.W

    def train_step(self, batch) -> torch.Tensor:
        if self._bstore is not None:
            return self._train_step_async(batch)
        if self._fused_ok():
            return self._train_step_fused(batch)
        return StaticStepMixin.train_step(self, batch)

    def _fused_ok(self) -> bool:
        """One worker on a GPU: every row of W is local, so the step is the two
        kernels of csrc/kernels/sparse_lr.hip (no dedup / routing / exchange).
        DTF_SLR_FUSED=0 keeps the general sharded path."""
        ok = getattr(self, "_fused", None)
        if ok is None:
            import os
            ok = self._fused = (self.world.world_size == 1 and self.device.type == "cuda" and self.W.dim == 1
                                and self.W.hogwild is None and self.W.router is None
                                and os.environ.get("DTF_SLR_FUSED", "1") != "0")
        return ok

    def _train_step_fused(self, batch) -> torch.Tensor:
        """Host batches (numpy arrays or CPU tensors) go through the plan's packed
        feed: one CSR pack into a pinned slot, one staging kernel, the two step
        kernels (SparseLRPlan.run_csr); device batches straight to the kernels."""
        labels, offsets, ids, vals = batch.to(self.device) if hasattr(batch, "to") else batch
        plan = getattr(self, "_plan", None)
        if plan is None:
            from .. import _native
            plan = self._plan = _native.load().SparseLRPlan(self.W.local, self.b.data, None)
        host = _host_arrays(labels, offsets, ids, vals)
        if host is not None and plan.run_csr(*host, self.lr):
            self.global_step += 1
            return plan.loss()
        dev = self.device
        loss = plan.step(_dev(labels, dev, torch.float32), _dev(offsets, dev, torch.int64),
                         _dev(ids, dev, torch.int64), None if vals is None else _dev(vals, dev, torch.float32),
                         self.lr)
        self.global_step += 1
        return loss

    def _train_step_async(self, batch) -> torch.Tensor:
        """One Hogwild step: pull b, rows straight from their owners, scatter-SGD
        into the owners' shards and `b -= lr g` in the shared store, no waiting."""
        self._bstore.pull()
        logits, labels, (rows, ctx) = self._forward(batch)
        loss = ops.sigmoid_xent(logits, labels)
        if self.b.grad is not None:
            self.b.grad = None
        loss.backward()
        g = rows.grad if rows.grad is not None else torch.zeros_like(rows)
        self.W.apply_sgd(ctx, g, self.lr)
        self.global_step = self._bstore.sgd_step([self.b.grad], self.lr)
        return loss.detach()

    def refresh_global_step(self) -> int:
        """Asynchronous mode: the shared step counter now (every worker's updates)."""
        if self._bstore is not None:
            self.global_step = self._bstore.global_step()
        return self.global_step

    def enable_graph(self, on: bool = True, example=None):
        """Replay each step as one captured hipGraph (GPU; needs the static
        device-resident routing: one worker, or an ids capacity for W > 1).
        With W > 1 every rank must call this at the same point: the capture
        runs the step's collectives (`example`: a batch of the training row
        count; default: an all-zero batch of `rows` rows)."""
        from ..utils.graphs import GraphedStep

        if not on:
            self._graphed = None
            return
        if self.device.type != "cuda" or (self.world.world_size > 1 and self.W.capacity is None):
            raise RuntimeError("graph capture needs a GPU and static routing (ids_capacity for W > 1)")
        strict = self.world.world_size > 1

        def step(labels, offsets, ids, vals):
            return self._train_step((labels, offsets, ids, vals))

        def state():
            st = [self.W.local, self.b.data]
            return st + (self.W.router.state() if self.W.router is not None else [])
        self._graphed = GraphedStep(step, state, strict=strict)
        self._example = self._static_batch(example if example is not None else self._zero_batch())
        if strict:
            self._graphed.capture(*self._example)

    def _zero_batch(self, rows: Optional[int] = None):
        rows = rows or self.rows
        n = self.W.capacity or rows
        per = max(1, n // rows)
        offsets = torch.clamp(torch.arange(rows + 1, dtype=torch.int64) * per, max=n)
        offsets[-1] = n
        return (torch.zeros(rows, 1), offsets, torch.zeros(n, dtype=torch.int64), torch.zeros(n))

    def _train_step(self, batch, exact: bool = False) -> torch.Tensor:
        logits, labels, (rows, ctx) = self._forward(batch, exact)
        loss = ops.sigmoid_xent(logits, labels)
        if self.b.grad is not None:
            self.b.grad = None
        loss.backward()
        ws = self.world.world_size
        g = rows.grad if rows.grad is not None else torch.zeros_like(rows)
        self.W.apply_sgd(ctx, g, self.lr / ws)
        with torch.no_grad():
            gb = self.b.grad.clone()
            if ws > 1:
                self.world.all_reduce(gb)
            if ctx.void is not None:          # a voided step changes nothing (replayed exactly later)
                gb *= (1 - ctx.void).to(gb.dtype)
            self.b -= (self.lr / ws) * gb
        return loss.detach()

    @torch.no_grad()
    def evaluate(self, batch):
        """(mean loss, probabilities) without updating (lr2.py Test(), :307-315).
        Lookups use the exact exchange: evaluation batches need no fixed shapes.
        Collective: first applies any voided steps of the current window."""
        self.sync_exchange()
        logits, labels, _ = self._forward(batch, exact=True)
        return ops.sigmoid_xent(logits, labels).detach(), torch.sigmoid(logits).reshape(-1)

    @torch.no_grad()
    def auc_update(self, batch):
        self.sync_exchange()
        logits, labels, _ = self._forward(batch, exact=True)
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
        """Collective: applies the voided steps of the current window first, so a
        checkpoint holds every batch trained so far."""
        self.sync_exchange()
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


def _dev(t, dev, dtype):
    if not torch.is_tensor(t):
        t = torch.as_tensor(t)
    return t.to(dev, dtype).contiguous()


def _host_arrays(labels, offsets, ids, vals):
    """numpy views (float32 labels / values, int64 offsets / ids) of a host
    batch, or None when any part is on a GPU."""
    out = []
    for t, dt in ((labels, np.float32), (offsets, np.int64), (ids, np.int64), (vals, np.float32)):
        if t is None:
            out.append(None)
            continue
        if torch.is_tensor(t):
            if t.device.type != "cpu":
                return None
            t = t.detach().numpy()
        out.append(np.asarray(t, dtype=dt))
    return out

