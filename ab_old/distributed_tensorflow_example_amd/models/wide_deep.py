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
Embedding rows use sparse SGD (the ps-side ScatterSub of TF) or TF's sparse
Adagrad / Momentum / RMSProp / Adam rules (`sparse_opt`, applied by the row
owner: ShardedEmbedding.set_optimizer), the tower uses SGD or TF-Adam
through the fused multi-tensor kernel.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from .. import ops, optim
from ..parallel.sharded_embedding import (ShardedEmbedding, StaticStepMixin, apply_sgd_shared, lookup_shared,
                                          pad_to_capacity)
from ..parallel.world import World, get_world


def _no_sink_hook(p):
    """grad_sink's readiness callback: the tower's bucket is reduced after backward."""


class WideDeep(StaticStepMixin):
    def __init__(self, num_features: int, emb_dim: int = 64, hidden: Sequence[int] = (256, 128),
                 lr: float = 0.05, dense_lr: Optional[float] = None, dense_opt: str = "sgd", combiner: str = "sum",
                 world: Optional[World] = None, seed: int = 1, device=None, emb_std: float = 0.05,
                 ids_capacity: Optional[int] = None, rows: int = 4096, peer_capacity: Optional[int] = None,
                 sparse_opt: str = "sgd", sparse_hp: Optional[dict] = None):
        self.world = world or get_world()
        self.device = torch.device(device) if device is not None else self.world.device
        self.lr = float(lr)
        self.combiner = combiner
        self.ids_capacity = ids_capacity   # per-batch id bound -> device-resident static routing
        if ids_capacity is not None and combiner != "sum":
            raise ValueError("static routing (ids_capacity) pads batches inside the last bag: 'sum' combiner only")
        # both tables route the same ids over the same partition: one router
        self.wide = ShardedEmbedding(num_features, 1, self.world, init_std=0.01, seed=seed, device=self.device,
                                     name="wide/weights", capacity=ids_capacity, peer_capacity=peer_capacity)
        self.emb = ShardedEmbedding(num_features, emb_dim, self.world, init_std=emb_std, seed=seed + 1,
                                    device=self.device, name="deep/embedding", capacity=ids_capacity,
                                    router=self.wide.router)
        # the tables' owner-side rule: sgd (TF ScatterSub) | adagrad | momentum | rmsprop | adam
        for t in (self.wide, self.emb):
            t.set_optimizer(sparse_opt, **(sparse_hp or {}))
        self.rows = int(rows)              # batch rows of the captured step
        self._window = []                  # static steps since the router's last check (replay source)
        self._example = None
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
            # the tower's backward kernels accumulate straight into these views
            # (ops/grad_sink.py: no zeroed temporaries, no AccumulateGrad adds);
            # flat_grad is zeroed once per step
            p._dtf_sink_hook = _no_sink_hook
            off += p.numel()
        dl = self.lr if dense_lr is None else float(dense_lr)
        self.opt = optim.FusedAdam(self.dense_params, dl) if dense_opt == "adam" else \
            optim.FusedSGD(self.dense_params, dl)
        if self.world.world_size > 1:
            with torch.no_grad():
                for p in self.dense_params:
                    self.world.broadcast(p.data, 0)
        self.comm_stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        if self.device.type == "cuda" and self.world.world_size > 1:
            # collective: the data plane of the tower's flat all-reduce (IPC on one
            # node, RCCL when it comes up for large towers), before the first step
            self.world.gpu_coll(self.flat_grad.numel() * self.flat_grad.element_size())
        self.global_step = 0
        self._graphed = None
        self._one = None

    def forward(self, labels, offsets, ids, vals, exact: bool = False):
        wide, h, extras = self.forward_parts(labels, offsets, ids, vals, exact)
        return wide + h + self.bias, extras

    def forward_parts(self, labels, offsets, ids, vals, exact: bool = False):
        """(wide part, tower output, (rows, rows, routing)) -- the logit is their
        sum + the shared bias."""
        # both tables read the same ids over the same row partition: one
        # dedup + id exchange, one row exchange carrying [U, 1 + D]
        ctx = self.wide.route(ids, capacity=self.ids_capacity, exact=exact)
        offsets = offsets.to(self.device).long()
        vals = None if vals is None else vals.to(self.device).float()
        if self.wide.W == 1 and self.device.type == "cuda" and not ctx.hogwild:
            # one GPU: the bags read the table rows in place (table[uniq[inverse]]); the
            # [U, D] row tensors are only the gradient targets (never gathered)
            U = ctx.uniq.numel()
            wrows = torch.empty((U, 1), device=self.device).requires_grad_(True)
            erows = torch.empty((U, self.emb.dim), device=self.device).requires_grad_(True)
            wide = ops.embedding_bag(wrows, ctx.inverse, offsets, vals, "sum", table=self.wide.local, remap=ctx.uniq)
            emb = ops.embedding_bag(erows, ctx.inverse, offsets, vals, self.combiner, table=self.emb.local,
                                    remap=ctx.uniq)
        else:
            wrows, erows = lookup_shared([self.wide, self.emb], ctx)
            wrows = wrows.detach().requires_grad_(True)
            erows = erows.detach().requires_grad_(True)
            wide = ops.embedding_bag(wrows, ctx.inverse, offsets, vals, "sum")
            emb = ops.embedding_bag(erows, ctx.inverse, offsets, vals, self.combiner)
        h = emb
        nl = len(self.layers) // 2
        for i in range(nl):
            h = ops.linear_act(h, self.layers[2 * i], self.layers[2 * i + 1], "relu" if i < nl - 1 else "none")
        return wide, h, (wrows, erows, ctx)

    def _static_batch(self, batch):
        labels, offsets, ids, vals = batch.to(self.device) if hasattr(batch, "to") else batch
        offsets = offsets.to(self.device).long()
        ids = ids.to(self.device)
        vals = None if vals is None else vals.to(self.device).float()
        self._last_empty = ids.numel() == 0
        if self.ids_capacity is not None:    # fixed shapes for the captured / static step
            offsets, ids, vals = pad_to_capacity(offsets, ids, vals, self.ids_capacity)
        return labels.to(self.device), offsets, ids, vals

    def _router(self):
        return self.wide.router

    def _route_table(self):
        return self.wide          # routes both tables' ids

    def enable_graph(self, on: bool = True, example=None):
        """Replay each training step as ONE captured hipGraph: routing, the two
        table lookups, bags, the MFMA tower, loss, backward, the sparse SGD of
        both tables and the fused Adam of the tower (~40 kernels) in one launch.
        Needs a GPU and the static device-resident routing (ids_capacity).  With
        W > 1 every rank calls this at the same point: the capture runs the
        step's collectives (`example`: a batch of the training row count;
        default an all-zero batch of `rows` rows)."""
        from ..utils.graphs import GraphedStep

        if not on:
            self._graphed = None
            return
        if self.device.type != "cuda" or self.ids_capacity is None:
            raise RuntimeError("graph capture needs a GPU and static routing (ids_capacity)")
        strict = self.world.world_size > 1

        def step(labels, offsets, ids, vals):
            return self._train_step((labels, offsets, ids, vals))

        def state():   # everything a step mutates, restored after the capture's warmup
            st = self.wide.state_tensors() + self.emb.state_tensors() + [p.data for p in self.dense_params]
            st += [self.opt.step_t]
            st += [t for t in list(self.opt.m) + list(self.opt.v) if t is not None]
            return st + (self.wide.router.state() if self.wide.router is not None else [])
        self._graphed = GraphedStep(step, state, strict=strict)
        self._example = self._static_batch(example if example is not None else self._zero_batch())
        if strict:
            self._graphed.capture(*self._example)

    def _zero_batch(self):
        rows, n = self.rows, self.ids_capacity
        per = max(1, n // rows)
        offsets = torch.clamp(torch.arange(rows + 1, dtype=torch.int64) * per, max=n)
        offsets[-1] = n
        return (torch.zeros(rows, 1), offsets, torch.zeros(n, dtype=torch.int64), torch.zeros(n))

    def _train_step(self, batch, exact: bool = False) -> torch.Tensor:
        labels, offsets, ids, vals = batch.to(self.device) if hasattr(batch, "to") else batch
        self.flat_grad.zero_()
        wide, h, (wrows, erows, lctx) = self.forward_parts(labels, offsets, ids, vals, exact)
        loss = ops.logit3_xent(wide, h, self.bias, labels)      # the head's adds + xent + mean: one kernel
        if self._one is None or self._one.device != loss.device:
            self._one = torch.ones((), device=loss.device)       # backward's seed, not a fill per step
        loss.backward(self._one)
        ws = self.world.world_size
        # dense tower: one flat all-reduce, overlapped with the sparse exchanges
        ev = None
        if ws > 1:
            coll = self.world.gpu_coll(self.flat_grad.numel() * self.flat_grad.element_size())
            if self.comm_stream is not None and coll is not None and coll is self.world.comm:
                # (RCCL: overlapped with the sparse exchanges on a side stream; the IPC
                # collectives keep one stream order, so they stay on this stream)
                self.comm_stream.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(self.comm_stream):
                    self.world.all_reduce(self.flat_grad)
                ev = torch.cuda.Event()
                ev.record(self.comm_stream)
            else:
                self.world.all_reduce(self.flat_grad)
        grads = [r.grad if r.grad is not None else torch.zeros_like(r) for r in (wrows, erows)]
        apply_sgd_shared([self.wide, self.emb], lctx, grads, [self.lr] * 2, grad_scale=1.0 / ws)
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)
        # a voided step (sharded exchange overflow on some rank) leaves the tower,
        # its Adam slots and step count untouched: decided on the device
        self.opt.step(grad_scale=1.0 / ws, skip=lctx.void)
        return loss.detach()

    @torch.no_grad()
    def predict(self, batch) -> torch.Tensor:
        self.sync_exchange()      # collective: the voided steps of the window are applied first
        labels, offsets, ids, vals = batch.to(self.device) if hasattr(batch, "to") else batch
        logit, _ = self.forward(labels, offsets, ids, vals, exact=True)
        return torch.sigmoid(logit).reshape(-1)

    def checkpoint_tensors(self):
        """(sharded, replicated) tensors under TF names.  Collective: applies the
        voided steps of the current window first.  Adam state is complete: the
        tower's slots (`<var>/Adam`, `<var>/Adam_1`) and `beta1_power` /
        `beta2_power` (TF's beta^(t+1) after t updates), and the tables' own
        sparse-Adam powers under `sparse/`."""
        self.sync_exchange()
        local = {self.wide.name: self.wide, self.emb.name: self.emb}   # TF partitioned variables
        for t in (self.wide, self.emb):                                 # their optimizer slots, sharded alike
            for sname in t.slots:
                local[f"{t.name}/{sname}"] = t.slot_view(sname)
        repl = {}
        for name, p, i in self._dense_names():
            repl[name] = p.detach()
            for sname, st in (("Adam", self.opt.m[i]), ("Adam_1", self.opt.v[i])):
                if st is not None:
                    repl[f"{name}/{sname}"] = st.detach()
        repl.update(self._powers("", self.opt))
        if self.wide._adam is not None:
            repl.update(self._powers("sparse/", self.wide._adam))
        repl["global_step"] = torch.tensor(self.global_step, dtype=torch.int64)
        return local, repl

    def _dense_names(self):
        names = []
        for i in range(len(self.layers) // 2):
            names += [f"deep/dense_{i}/kernel", f"deep/dense_{i}/bias"]
        names.append("bias")
        return [(n, p, i) for i, (n, p) in enumerate(zip(names, self.dense_params))]

    @staticmethod
    def _powers(prefix, opt):
        if opt.kind not in ("adam", "adamw"):
            return {}
        t = int(opt.step_t.item())
        # the integer count itself rides along (`adam_step`): the float32 powers
        # underflow (beta1 = 0.9: 0.0 after ~990 steps) and cannot pin it alone
        return {f"{prefix}beta1_power": torch.tensor(opt.b1 ** (t + 1), dtype=torch.float32),
                f"{prefix}beta2_power": torch.tensor(opt.b2 ** (t + 1), dtype=torch.float32),
                f"{prefix}adam_step": torch.tensor(t, dtype=torch.int64)}

    def restore(self, prefix: str):
        """Load a checkpoint written from `checkpoint_tensors` (any world size):
        tables and slots take the rows they own, the tower, its Adam slots and
        every optimizer's step count (the saved `adam_step`; a checkpoint without
        it: from both beta powers, `optim.adam_steps_from_powers`) are restored."""
        from ..ckpt import read_bundle_index, read_tensor, restore_sharded
        from ..optim import adam_steps_from_powers

        local, repl = self.checkpoint_tensors()
        idx = read_bundle_index(prefix)
        restore_sharded(prefix, {k: v for k, v in local.items()})
        with torch.no_grad():
            for name, dst in repl.items():
                if name.endswith(("beta2_power", "adam_step")) or name == "global_step":
                    continue
                if name.endswith("beta1_power"):
                    pre = name[: -len("beta1_power")]
                    opt = self.opt if pre == "" else self.wide._adam
                    if pre + "adam_step" in idx:
                        steps = int(read_tensor(prefix, pre + "adam_step"))
                    elif name in idx:
                        b2 = float(read_tensor(prefix, pre + "beta2_power")) if pre + "beta2_power" in idx else None
                        steps = adam_steps_from_powers(float(read_tensor(prefix, name)), opt.b1, b2, opt.b2)
                    else:
                        continue
                    opts = [opt] if opt is self.opt else [self.wide._adam, self.emb._adam]
                    for o in opts:
                        o.step_t.fill_(steps)
                    continue
                if name in idx:          # dst shares storage with the parameter / slot
                    dst.copy_(read_tensor(prefix, name).to(self.device, torch.float32).reshape(dst.shape))
        if "global_step" in idx:
            self.global_step = int(read_tensor(prefix, "global_step"))
