"""Wide & Deep CTR model with PS-style sharded embedding tables (BASELINE #5).

Grows out of the reference's sparse LR (lr2.py:368-396, the *wide* part)
and its commented deep tower (lr2_debug.py:423-428: `deep_w1[F,128]` via
embedding_lookup_sparse, `deep_w2[128,1]`, `py_x += deep_h2`).

    wide  = sum_j W_wide[id_j] * val_j + b                 (sharded [F, 1])
    emb   = combine_j E[id_j] * val_j   (sum | mean)       (sharded [F, D])
    deep  = MLP(emb): D -> h1 -> h2 -> 1, ReLU             (replicated, MFMA linear_act)
    logit = wide + deep ;  loss = mean sigmoid_xent(logit, y)

MI355X mapping: both tables are row-sharded over all GPUs (the ps role of
replica_device_setter, one shard per rank, all-to-all lookups/updates
sized for 288 GB HBM per shard); the dense tower is replicated and its
gradients travel in one flat bucket all-reduce (RCCL over xGMI) that is
launched on a side stream while the sparse all-to-all updates run.
Embedding rows use sparse SGD (the ps-side ScatterSub of TF), the tower
uses SGD or TF-Adam through the fused multi-tensor kernel.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from .. import ops, optim
from ..parallel.sharded_embedding import ShardedEmbedding, apply_sgd_shared, lookup_shared
from ..parallel.world import World, get_world


class WideDeep:
    def __init__(self, num_features: int, emb_dim: int = 64, hidden: Sequence[int] = (256, 128),
                 lr: float = 0.05, dense_lr: Optional[float] = None, dense_opt: str = "sgd", combiner: str = "sum",
                 world: Optional[World] = None, seed: int = 1, device=None, emb_std: float = 0.05,
                 ids_capacity: Optional[int] = None):
        self.world = world or get_world()
        self.device = torch.device(device) if device is not None else self.world.device
        self.lr = float(lr)
        self.combiner = combiner
        self.ids_capacity = ids_capacity   # per-batch id bound -> device-resident static routing
        self.wide = ShardedEmbedding(num_features, 1, self.world, init_std=0.01, seed=seed, device=self.device,
                                     name="wide/weights")
        self.emb = ShardedEmbedding(num_features, emb_dim, self.world, init_std=emb_std, seed=seed + 1,
                                    device=self.device, name="deep/embedding")
        g = torch.Generator().manual_seed(seed + 2)
        dims = [emb_dim] + list(hidden) + [1]
        self.layers: List[torch.nn.Parameter] = []
        for i in range(len(dims) - 1):
            w = torch.randn(dims[i], dims[i + 1], generator=g) * (2.0 / dims[i]) ** 0.5
            self.layers += [torch.nn.Parameter(w.to(self.device)),
                            torch.nn.Parameter(torch.zeros(dims[i + 1], device=self.device))]
        self.bias = torch.nn.Parameter(torch.zeros(1, device=self.device))
        self.dense_params = self.layers + [self.bias]
        n = sum(p.numel() for p in self.dense_params)
        self.flat_grad = torch.zeros(n, dtype=torch.float32, device=self.device)
        off = 0
        for p in self.dense_params:                   # grads are views of one bucket
            p.grad = self.flat_grad[off:off + p.numel()].view_as(p)
            off += p.numel()
        dl = self.lr if dense_lr is None else float(dense_lr)
        self.opt = optim.FusedAdam(self.dense_params, dl) if dense_opt == "adam" else \
            optim.FusedSGD(self.dense_params, dl)
        if self.world.world_size > 1:
            with torch.no_grad():
                for p in self.dense_params:
                    self.world.broadcast(p.data, 0)
        self.comm_stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self.global_step = 0
        self._graphed = None

    def forward(self, labels, offsets, ids, vals):
        # both tables read the same ids over the same row partition: one
        # dedup + id exchange, one row exchange carrying [U, 1 + D]
        ctx = self.wide.route(ids, capacity=self.ids_capacity)
        wrows, erows = lookup_shared([self.wide, self.emb], ctx)
        wrows = wrows.detach().requires_grad_(True)
        erows = erows.detach().requires_grad_(True)
        offsets = offsets.to(self.device).long()
        vals = None if vals is None else vals.to(self.device).float()
        wide = ops.embedding_bag(wrows, ctx.inverse, offsets, vals, "sum")
        emb = ops.embedding_bag(erows, ctx.inverse, offsets, vals, self.combiner)
        h = emb
        nl = len(self.layers) // 2
        for i in range(nl):
            h = ops.linear_act(h, self.layers[2 * i], self.layers[2 * i + 1], "relu" if i < nl - 1 else "none")
        logit = wide + h + self.bias
        return logit, (wrows, erows, ctx)

    def train_step(self, batch) -> torch.Tensor:
        if self._graphed is not None:
            labels, offsets, ids, vals = batch.to(self.device) if hasattr(batch, "to") else batch
            loss = self._graphed(labels, offsets, ids, vals)
            self.global_step += 1
            return loss.detach()
        return self._train_step(batch)

    def enable_graph(self, on: bool = True):
        """Replay each training step as ONE captured hipGraph: routing, the two
        table lookups, bags, the MFMA tower, loss, backward, the sparse SGD of
        both tables and the fused Adam of the tower (~40 kernels) in one launch.
        Needs a GPU and the static device-resident routing (ids_capacity)."""
        from ..utils.graphs import GraphedStep

        if not on:
            self._graphed = None
            return
        if self.device.type != "cuda" or self.ids_capacity is None:
            raise RuntimeError("graph capture needs a GPU and static routing (ids_capacity)")

        def step(labels, offsets, ids, vals):
            gs = self.global_step
            loss = self._train_step((labels, offsets, ids, vals))
            self.global_step = gs          # counted by train_step, not by warmup/capture
            return loss

        def state():   # everything a step mutates, restored after the capture's warmup
            st = [self.wide.local, self.emb.local] + [p.data for p in self.dense_params] + [self.opt.step_t]
            st += [t for t in list(self.opt.m) + list(self.opt.v) if t is not None]
            return st
        self._graphed = GraphedStep(step, state)

    def _train_step(self, batch) -> torch.Tensor:
        labels, offsets, ids, vals = batch.to(self.device) if hasattr(batch, "to") else batch
        self.flat_grad.zero_()
        logit, (wrows, erows, lctx) = self.forward(labels, offsets, ids, vals)
        loss = ops.sigmoid_xent(logit, labels)
        loss.backward()
        ws = self.world.world_size
        # dense tower: one flat all-reduce, overlapped with the sparse exchanges
        ev = None
        if ws > 1:
            if self.comm_stream is not None and self.world.comm is not None:
                self.comm_stream.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(self.comm_stream):
                    self.world.all_reduce(self.flat_grad)
                ev = torch.cuda.Event()
                ev.record(self.comm_stream)
            else:
                self.world.all_reduce(self.flat_grad)
        grads = [r.grad if r.grad is not None else torch.zeros_like(r) for r in (wrows, erows)]
        apply_sgd_shared([self.wide, self.emb], lctx, grads, [self.lr / ws] * 2)
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)
        self.opt.step(grad_scale=1.0 / ws)
        self.global_step += 1
        return loss.detach()

    @torch.no_grad()
    def predict(self, batch) -> torch.Tensor:
        labels, offsets, ids, vals = batch.to(self.device) if hasattr(batch, "to") else batch
        logit, _ = self.forward(labels, offsets, ids, vals)
        return torch.sigmoid(logit).reshape(-1)

    def checkpoint_tensors(self):
        local = {self.wide.name: self.wide, self.emb.name: self.emb}   # TF partitioned variables
        names = []
        for i in range(len(self.layers) // 2):
            names += [f"deep/dense_{i}/kernel", f"deep/dense_{i}/bias"]
        repl = {n: p.detach() for n, p in zip(names, self.layers)}
        repl["bias"] = self.bias.detach()
        repl["global_step"] = torch.tensor(self.global_step, dtype=torch.int64)
        return local, repl
