"""Row-sharded embedding tables: the parameter-server role, one shard per GPU.

Reference: the LR weight `W[F, 1]` (F = 4.7M, 1e9 in product,
lr2.py:384 / run_lr2.sh:56) lives on ps0 via replica_device_setter
(lr2.py:359-361); each step the worker sends the batch's unique ids, the ps
gathers rows, the worker returns IndexedSlices gradients that the ps
scatter-applies.  The commented Wide&Deep tower
(lr2_debug.py:423-428) adds a [F, 128] table the same way.

MI355X design: row r lives on rank r % W at local row r // W (288 GB of
HBM per GPU holds a 1e9 x 1 fp32 shard 8x over).  Per step:

  lookup:  dedup ids (torch.unique) -> bucket by owner -> all-to-all of ids
           -> owners gather rows -> all-to-all back            (RCCL / gloo)
  combine: the CSR bag kernel (ops.embedding_bag) runs over the gathered
           [U, D] block with ids remapped to 0..U-1
  update:  bag backward into a dense [U, D] gradient -> all-to-all to owners
           -> owners apply SGD with the fused scatter kernel

Each row has exactly one owner, so there is no replica drift and no
all-reduce of a dense F x D gradient.

Static (capturable) routing: with an ids-per-batch bound the exchange is an
equal-split all-to-all of `peer_cap` id slots per peer, decided on the device
(no host read-back).  `peer_cap` is right-sized to the owners' measured
unique-id load (a `StaticRouter` tracks the all-reduced peak per owner and
resizes every `check_every` steps, identically on every rank), so the padded
exchange moves ~slack x the exact bytes instead of the whole batch per peer.
A batch whose ids overflow an owner's slots on ANY rank is VOIDED on every
rank (the all-reduced flag zeroes the sparse gradients and skips the dense
updates on the device), and so is every later batch of the check window; the
check replays them in their original order through the exact exchange --
deterministic, identical on all ranks, the same updates as a synchronous run,
never a silent drop.

Initial values are a counter-based (Philox4x32-10) normal of the *global* element index, generated on the device
by one kernel, so a table is bit-identical for any world size.
Checkpoints store the table as a TF partitioned variable (contiguous
fixed_size_partitioner slices, see ckpt/__init__.py).
"""
from __future__ import annotations

import copy
from typing import Optional

import torch

from .. import ops
from .world import World, get_world


class LookupCtx:
    """Routing of one batch.  Dynamic: exact per-peer counts (host lists in
    send/recv), `order` sorts uniq by owner.  Static: every peer gets `cap`
    slots (the router's per-peer capacity, identical on all ranks), `order`
    holds each unique id's slot (dest, -1 for padding / overflow) and uniq /
    recv_local carry -1 padding -- no host read-back, every shape fixed by the
    batch shape and the capacity.  `void`: device int32 [1], 1 when this step
    overflowed on some rank (static W > 1 only)."""
    __slots__ = ("uniq", "inverse", "order", "send", "recv", "recv_local", "static", "n", "void", "hogwild")

    def __init__(self, uniq, inverse, order, send, recv, recv_local, static=False, n=0, void=None, hogwild=False):
        self.uniq, self.inverse, self.order = uniq, inverse, order
        self.send, self.recv, self.recv_local = send, recv, recv_local
        self.static, self.n, self.void = static, n, void
        self.hogwild = hogwild      # rows read from the owners' shared shards (asynchronous mode)


class StaticRouter:
    """Per-peer capacity and overflow bookkeeping of the static exchange, shared
    by the tables that route the same ids (W&D's wide and deep tables).

    Device state (all mutated inside captured steps, so they are part of a
    GraphedStep's snapshot): `void` [1] int32 (this step's all-reduced
    overflow flag), `peak` [1] int64 (all-reduced max unique ids of one owner
    since the last check), `exact` [1] int64 (ids this rank would have sent in
    an exact exchange since the last check), `log` [K] int32 (the void flag of
    each step of the window), `pos` [1] int64 (step index in the window)."""

    def __init__(self, world: World, device, n_cap: int, peer_cap: Optional[int] = None, slack: float = 1.1,
                 check_every: int = 32, first_check: int = 4, align: int = 32):
        self.world, self.W = world, world.world_size
        self.device = torch.device(device)
        self.n_cap = int(n_cap)
        self.slack, self.align = float(slack), int(align)
        self.check_every, self.first_check = int(check_every), int(first_check)
        # start from a safe share of the batch (right-sized at the first check)
        self.peer_cap = int(peer_cap) if peer_cap is not None else self._round(-(-self.n_cap // max(1, self.W)))
        self.fixed = peer_cap is not None
        self.void = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.peak = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.exact = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.log = torch.zeros(max(self.check_every, self.first_check), dtype=torch.int32, device=self.device)
        self.pos = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.steps = 0                 # host: steps since the last check
        self.checks = self.resizes = self.voided = 0
        self.last_ratio = None         # host: static id slots / exact ids of the last checked window

    def _round(self, n: int) -> int:
        a = self.align
        return max(a, -(-int(n) // a) * a)

    def state(self):
        return [self.void, self.peak, self.exact, self.log, self.pos]

    def record(self, ocnt: torch.Tensor, rank: int):
        """Device-side bookkeeping of one static step (capturable): all-reduce
        [overflow, peak] (max) so every rank voids the same steps and resizes to
        the same capacity; log the void flag at the window position."""
        mx = ocnt.max().to(torch.int64)
        stat = torch.stack([(mx > self.peer_cap).to(torch.int64), mx])
        self.world.all_reduce(stat, "max")
        # sticky until the check: once a step is voided every later step of the
        # window is too, so the replay applies them all in their original order
        # (exact synchronous-SGD semantics, not a reordering)
        torch.maximum(self.void, stat[:1].to(torch.int32), out=self.void)
        torch.maximum(self.peak, stat[1:2], out=self.peak)
        self.exact += ocnt.sum().to(torch.int64) - ocnt[rank].to(torch.int64)
        self.log.index_copy_(0, self.pos % self.log.numel(), self.void)
        self.pos += 1

    def due(self) -> bool:
        lim = self.first_check if self.checks == 0 else self.check_every
        return self.steps >= min(lim, self.log.numel())

    def check(self):
        """Host side, every `check_every` steps (ONE sync): the window's void
        flags (positions to replay exactly) and the all-reduced peak; resize the
        per-peer capacity to slack x peak (identical on all ranks).  Returns
        (voided window positions, capacity changed)."""
        n = self.steps
        flags = self.log[:n].cpu().tolist() if n else []
        peak = int(self.peak.item())
        exact = int(self.exact.item())
        if n and exact:
            self.last_ratio = n * (self.W - 1) * self.peer_cap / exact
        self.log.zero_()
        self.pos.zero_()
        self.void.zero_()
        self.peak.zero_()
        self.exact.zero_()
        self.steps = 0
        self.checks += 1
        voided = [i for i, f in enumerate(flags) if f]
        self.voided += len(voided)
        changed = False
        if not self.fixed and peak > 0:
            want = self._round(self.slack * peak)
            # grow at once; shrink only when oversized by > 10 % (no resize churn)
            if want > self.peer_cap or want < 0.9 * self.peer_cap:
                self.peer_cap = want
                self.resizes += 1
                changed = True
        return voided, changed

    def wire_ratio(self) -> Optional[float]:
        """Id slots the static exchange sent to peers per id an exact exchange
        would have sent, over the last checked window (rows and gradients travel
        in the same slots, so this is the byte ratio of all three all-to-alls)."""
        return self.last_ratio


class ShardedEmbedding:
    def __init__(self, num_rows: int, dim: int = 1, world: Optional[World] = None, init_std: float = 1.0,
                 seed: int = 0, device=None, name: str = "embedding", zero_init: bool = False,
                 capacity: Optional[int] = None, peer_capacity: Optional[int] = None,
                 router: Optional[StaticRouter] = None):
        self.world = world or get_world()
        self.W = self.world.world_size
        self.rank = self.world.rank
        self.num_rows, self.dim, self.name = int(num_rows), int(dim), name
        self.capacity = capacity          # ids per batch bound (same on every rank) -> static routing
        self.device = torch.device(device) if device is not None else self.world.device
        # the static exchange's per-peer capacity + overflow bookkeeping (shared by
        # tables that route the same ids: pass the first table's router)
        self.router = router if router is not None else (
            StaticRouter(self.world, self.device, capacity, peer_capacity) if capacity is not None else None)
        # asynchronous (Hogwild) mode: every shard mapped into every rank
        # (parallel/async_ps.HogwildTable); lookups / updates bypass the exchange
        self.hogwild = None
        # owner-side update rule of the sparse gradients (set_optimizer)
        self.opt_kind, self.opt_hp, self.slots = "sgd", {}, {}
        self._gacc = None
        self._adam = None
        self._defer = None               # pending (row index) tensors of a multi-lookup sparse update
        self._empty = None               # device int32 [1]: this step's batch has no ids (set_batch_empty)
        n_local = (self.num_rows - self.rank + self.W - 1) // self.W if self.rank < self.num_rows else 0
        self.local = torch.empty((n_local, self.dim), dtype=torch.float32, device=self.device)
        with torch.no_grad():
            if zero_init:
                self.local.zero_()
            else:
                # local row i is global row i*W + rank: one counter-based
                # Philox kernel over the shard (csrc/kernels/random.hip)
                ops.philox_normal_(self.local, self.W, self.rank, seed, 0.0, init_std)

    # ------------------------------------------------------------------ exchange
    def route(self, ids: torch.Tensor, capacity: Optional[int] = None, exact: bool = False) -> LookupCtx:
        """Dedup `ids` and send each owner the unique ids it serves (no rows yet).

        The context depends only on the ids and the row partition, so tables
        with the same row count and world share it (`lookup_shared`).
        `capacity`: ids-per-batch bound configured identically on every rank ->
        the device-resident static exchange (no host read-back); without it
        (W > 1) the exact per-peer counts are exchanged and read on the host."""
        ids = ids.to(self.device).long()
        N = ids.numel()
        capacity = self.capacity if capacity is None else capacity
        if exact and self.W > 1:
            capacity = None          # the exact exchange (replays of voided steps)
        if N > 0 and (self.W == 1 or (capacity is not None and self.W <= _max_route_world())):
            if self.W > 1 and N > capacity:
                raise ValueError(f"{self.name}: batch has {N} ids, above the routing capacity {capacity}")
            if capacity is not None and self.W > 1 and self.router is not None and self.router.n_cap != capacity:
                raise ValueError(f"{self.name}: routing capacity {capacity} != the router's {self.router.n_cap}")
            return self._route_static(ids, int(capacity) if capacity is not None else N)
        if ids.is_cuda and 0 < N and self.num_rows < 2 ** 31:
            # one int32 radix sort serves both the dedup and (handed over to
            # ops) the sorted-segment backward of every bag over these ids
            sids, perm = torch.sort(ids.to(torch.int32))
            uniq32, inv_sorted = torch.unique_consecutive(sids, return_inverse=True)
            uniq = uniq32.long()
            inverse = torch.empty_like(ids)
            inverse[perm] = inv_sorted
            ops.register_sorted_ids(inverse, inv_sorted, perm)
        else:
            uniq, inverse = torch.unique(ids, return_inverse=True)
        if self.W == 1:
            return LookupCtx(uniq, inverse, None, None, None, uniq)
        owner = uniq % self.W
        order = torch.argsort(owner, stable=True)
        uniq_sorted = uniq[order]
        if self._empty is not None and bool(self._empty.item()):
            uniq_sorted = torch.full_like(uniq_sorted, -1)   # padding of an empty batch: no row is touched
        send = torch.bincount(owner, minlength=self.W)
        recv = torch.empty_like(send)
        self.world.all_to_all(send, [1] * self.W, recv, [1] * self.W)
        send_l, recv_l = send.tolist(), recv.tolist()
        recv_ids = torch.empty(sum(recv_l), dtype=torch.int64, device=self.device)
        self.world.all_to_all(uniq_sorted, send_l, recv_ids, recv_l)
        return LookupCtx(uniq, inverse, order, send_l, recv_l, recv_ids // self.W)

    def _route_static(self, ids: torch.Tensor, cap: int) -> LookupCtx:
        """Device-resident routing: radix sort + one dedup/bucketing kernel
        (csrc/kernels/sparse_route.hip) + an equal-split all-to-all of the
        router's per-peer capacity.  Nothing is read back to the host; an owner
        overflow voids the step on every rank (StaticRouter)."""
        N, W = ids.numel(), self.W
        small = self.num_rows < 2 ** 31
        sids, perm = torch.sort(ids.to(torch.int32) if small else ids)
        router = self.router
        if W > 1 and router is None:
            router = self.router = StaticRouter(self.world, self.device, cap)
        pc = router.peer_cap if W > 1 else N
        if ids.is_cuda:
            inv_sorted, inverse, uniq, dest, send, _count, ocnt = ops._C().sparse_route(sids.contiguous(), perm, W, pc)
            ops.register_sorted_ids(inverse, inv_sorted, perm)
        else:
            inv_sorted, inverse, uniq, dest, send, ocnt = _route_static_torch(sids, perm, W, pc)
        if self._empty is not None:
            # an empty batch is all padding: no id is sent or looked up as a
            # touched row (capturable: the flag is read on the device)
            e = self._empty.bool()
            uniq = uniq.masked_fill(e, -1)
            if W > 1:
                send = send.masked_fill(e, -1)
                dest = dest.masked_fill(e, -1)
                ocnt = ocnt.masked_fill(e, 0)
        if W == 1:
            return LookupCtx(uniq, inverse, None, None, None, uniq, static=True, n=N)
        router.record(ocnt, self.rank)
        recv = torch.empty(W * pc, dtype=torch.int64, device=self.device)
        self.world.all_to_all(send, [pc] * W, recv, [pc] * W)
        recv_local = torch.where(recv >= 0, recv // W, torch.full_like(recv, -1))
        return LookupCtx(uniq, inverse, dest.long(), [pc] * W, [pc] * W, recv_local, static=True, n=pc,
                         void=router.void)

    def lookup(self, ids: torch.Tensor):
        """rows [U, D] for the unique ids of `ids`, plus the routing context."""
        if self.hogwild is not None:      # asynchronous: straight from the owners' shards, no collective
            rows, inverse, uniq = self.hogwild.lookup(ids)
            return rows, LookupCtx(uniq, inverse, None, None, None, None, hogwild=True)
        # outside a training step: the exact exchange (the static one records
        # into the router's per-step window, which only train steps advance)
        ctx = self.route(ids, exact=True)
        return lookup_shared([self], ctx)[0], ctx

    def apply_sgd(self, ctx: LookupCtx, grad_rows: torch.Tensor, lr: float, grad_scale: float = 1.0):
        """The owner-side update of the rows of ctx.uniq (grad_rows aligned with
        it): `local[rows] -= lr * grad_scale * grad` with the default SGD rule,
        else the rule of `set_optimizer`."""
        if ctx.hogwild:
            if self.opt_kind != "sgd":
                raise NotImplementedError("asynchronous (Hogwild) table updates: SGD only")
            self.hogwild.scatter_sgd(ctx.uniq, grad_rows, lr * grad_scale)
            return
        apply_sgd_shared([self], ctx, [grad_rows], [lr], grad_scale)

    # ------------------------------------------------------------------ optimizer
    def set_optimizer(self, kind: str = "sgd", **hp):
        """The owner-side update of this table's sparse gradients, TensorFlow's
        sparse-apply semantics (duplicates summed, then each touched row):

          sgd       var -= lr g                                  (ScatterSub / SparseApplyGradientDescent)
          momentum  acc = mu acc + g; var -= lr acc (nesterov)   slot Momentum   (hp: momentum, use_nesterov)
          adagrad   acc += g^2; var -= lr g / sqrt(acc)          slot Adagrad    (hp: initial_accumulator_value)
          rmsprop   ms / mom as tf.train.RMSPropOptimizer        slots RMSProp, Momentum (hp: decay, momentum, epsilon)
          adam      tf.train.AdamOptimizer's _apply_sparse: m, v decay on EVERY row of the shard,
                    the step moves every row (dense over the shard)  slots Adam, Adam_1 (hp: beta1, beta2, epsilon)

        Row-local rules run one kernel over the step's touched rows
        (csrc/kernels/sparse_optim.hip); Adam runs the fused multi-tensor Adam
        over the shard.  Slots are sharded like the table (`slot_view`)."""
        if kind not in ("sgd", "momentum", "adagrad", "rmsprop", "adam"):
            raise ValueError(f"{self.name}: no sparse update rule '{kind}'")
        if kind == self.opt_kind and hp == self.opt_hp:
            return
        self.opt_kind, self.opt_hp = kind, dict(hp)
        self.slots, self._adam = {}, None
        z = torch.zeros_like(self.local)
        if kind == "momentum":
            self.slots["Momentum"] = z
        elif kind == "adagrad":
            self.slots["Adagrad"] = z.fill_(float(hp.get("initial_accumulator_value", 0.1)))
        elif kind == "rmsprop":
            self.slots["RMSProp"] = torch.ones_like(self.local)
            self.slots["Momentum"] = z
        elif kind == "adam":
            from .. import optim
            self._adam = optim.FusedAdam([self.local], 0.001, float(hp.get("beta1", 0.9)),
                                         float(hp.get("beta2", 0.999)), float(hp.get("epsilon", 1e-8)))
            self.slots["Adam"], self.slots["Adam_1"] = self._adam.m[0], self._adam.v[0]
        self._empty = None if kind == "sgd" else torch.zeros(1, dtype=torch.int32, device=self.device)
        # [local rows + 1 dump row] accumulator of a step's summed gradients, zero between steps
        self._gacc = None if kind == "sgd" else torch.zeros((self.local.shape[0] + 1, self.dim),
                                                            dtype=torch.float32, device=self.device)

    def set_batch_empty(self, empty: bool):
        """Mark the next routed batch as empty (all padding).  Only matters for
        the row-local sparse rules: TF touches no row on an empty batch, while
        the static padding would repeat id 0 with a zero gradient (SGD: a
        no-op, so nothing is recorded)."""
        if self.opt_kind == "sgd" and self._empty is None:
            return
        if self._empty is None:
            self._empty = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._empty.fill_(1 if empty else 0)

    def begin_update(self):
        """Collect the sparse gradients of several lookups of this table into one
        update (TF sums the IndexedSlices of every lookup, then applies the rule
        once): `apply_sgd` calls only accumulate until `finish_update`."""
        if self.opt_kind != "sgd":
            self._defer = []

    def finish_update(self, lr: float, void: Optional[torch.Tensor] = None):
        pend, self._defer = self._defer, None
        if pend:
            self._apply_rule(torch.cat(pend), lr, void)

    def slot_view(self, slot: str) -> "ShardedEmbedding":
        """The slot as a table of the same geometry (checkpoint save / restore)."""
        v = copy.copy(self)
        v.local, v.name = self.slots[slot], f"{self.name}/{slot}"
        v.router, v.hogwild, v.slots, v.opt_kind, v._gacc, v._adam = None, None, {}, "sgd", None, None
        v._defer, v._empty = None, None
        return v

    def state_tensors(self):
        """Everything an update mutates (graph-capture warmup save / restore)."""
        st = [self.local] + list(self.slots.values())
        return st + ([self._adam.step_t] if self._adam is not None else [])

    def _sgd_local(self, ctx: LookupCtx, g: torch.Tensor, lr: float, grad_scale: float = 1.0,
                   void: Optional[torch.Tensor] = None):
        n = g.shape[0]
        if n == 0:
            return
        if self.opt_kind != "sgd":
            self._apply_local(ctx.recv_local, g, lr, grad_scale, void)
            return
        with torch.no_grad():      # one gradient row per id: no offsets tensor
            ops.embedding_bag_sgd_(self.local, ctx.recv_local, None, None, g, float(lr) * grad_scale)

    @torch.no_grad()
    def _apply_local(self, idx: torch.Tensor, g: torch.Tensor, lr: float, grad_scale: float,
                     void: Optional[torch.Tensor]):
        """idx[i]: local row of gradient row i (-1: padding); rows may repeat
        (several ranks looked the same row up).  Fixed shapes throughout -- no
        host read-back, so the update is capturable."""
        nl = self.local.shape[0]
        i = torch.where(idx >= 0, idx, torch.full_like(idx, nl))
        self._gacc.index_add_(0, i, g if grad_scale == 1.0 else g * grad_scale)
        if self._defer is not None:        # more lookups of this table follow in this step
            self._defer.append(i)
            return
        self._apply_rule(i, lr, void)

    @torch.no_grad()
    def _apply_rule(self, i: torch.Tensor, lr: float, void: Optional[torch.Tensor]):
        """The rule over the rows accumulated in _gacc (i: their local indices,
        nl = the dump row of padding), then clear them."""
        nl = self.local.shape[0]
        s, _ = torch.sort(i)
        hp = self.opt_hp
        if self.opt_kind == "adam":
            self._adam.set_lr(lr)
            self._adam.step([self._gacc[:nl]], skip=void)
        else:
            head = torch.ones_like(s, dtype=torch.bool)
            head[1:] = s[1:] != s[:-1]
            rows = torch.where(head & (s < nl), s, torch.full_like(s, -1))    # each touched row once
            gsum = self._gacc.index_select(0, s)
            kind = {"momentum": 1, "adagrad": 4, "rmsprop": 5}[self.opt_kind]
            sa = self.slots.get("Adagrad", self.slots.get("RMSProp", self.slots.get("Momentum")))
            sb = self.slots.get("Momentum") if self.opt_kind == "rmsprop" else None
            mu = float(hp.get("momentum", 0.0))
            args = (kind, float(lr), mu, bool(hp.get("use_nesterov", False)), float(hp.get("decay", 0.9)),
                    float(hp.get("epsilon", 1e-10)))
            if self.local.is_cuda:
                ops._C().sparse_rows_apply(self.local, sa, sb, rows, gsum, *args,
                                           skip=None if void is None else void.reshape(-1)[:1].to(torch.int32))
            else:
                _rows_apply_torch(self.local, sa, sb, rows, gsum, *args, skip=void)
        self._gacc.index_fill_(0, s, 0.0)

    # ------------------------------------------------------------------ bags
    def bag_forward(self, ids, offsets, weights=None, mode: str = "sum"):
        """embedding_lookup_sparse over the sharded table -> ([B, D], ctx)."""
        rows, ctx = self.lookup(ids)
        rows = rows.detach().requires_grad_(True)
        out = ops.embedding_bag(rows, ctx.inverse, offsets.to(self.device).long(),
                                None if weights is None else weights.to(self.device).float(), mode)
        return out, (rows, ctx)

    def bag_backward_sgd(self, state, lr: float):
        rows, ctx = state
        g = rows.grad if rows.grad is not None else torch.zeros_like(rows)
        self.apply_sgd(ctx, g, lr)

    # ------------------------------------------------------------------ checkpoint
    def full_table(self) -> torch.Tensor:
        """Gather the whole table on every rank (small tables / tests only)."""
        if self.W == 1:
            return self.local.detach().clone()
        n_max = (self.num_rows + self.W - 1) // self.W
        pad = torch.zeros((n_max, self.dim), dtype=torch.float32, device=self.device)
        pad[: self.local.shape[0]] = self.local
        allp = torch.empty((self.W * n_max, self.dim), dtype=torch.float32, device=self.device)
        self.world.all_gather(pad, allp)
        allp = allp.view(self.W, n_max, self.dim)
        out = torch.empty((self.num_rows, self.dim), dtype=torch.float32, device=self.device)
        for r in range(self.W):
            n_r = (self.num_rows - r + self.W - 1) // self.W
            out[r::self.W] = allp[r, :n_r]
        return out

    def shard_name(self) -> str:
        return f"{self.name}/part_{self.rank}"

    def load_full(self, table: torch.Tensor):
        with torch.no_grad():
            self.local.copy_(table.to(self.device)[self.rank::self.W])


def _check_shared(tables):
    t0 = tables[0]
    for t in tables[1:]:
        if t.num_rows != t0.num_rows or t.world is not t0.world:
            raise ValueError("tables sharing one routing context need the same row count and world")


def lookup_shared(tables, ctx: LookupCtx):
    """Rows of every table for ctx.uniq with ONE row all-to-all: owners gather
    each table's rows side by side ([n, sum D]) so W&D's wide and deep tables
    (same ids, same partition) pay one dedup, one id exchange and one row
    exchange per step instead of two of each."""
    _check_shared(tables)
    t0 = tables[0]
    if t0.W == 1:
        idx = ctx.uniq.clamp_min(0) if ctx.static else ctx.uniq     # padding slots read row 0, never used
        return [t.local.index_select(0, idx) for t in tables]
    dims = [t.dim for t in tables]
    src = ctx.recv_local.clamp_min(0)           # -1: padding slots / an empty batch's ids, never used
    served = torch.cat([t.local.index_select(0, src) for t in tables], 1) if len(tables) > 1 else \
        t0.local.index_select(0, src)
    got = torch.empty((sum(ctx.send), sum(dims)) if ctx.static else (ctx.uniq.numel(), sum(dims)),
                      dtype=torch.float32, device=t0.device)
    t0.world.all_to_all(served.contiguous(), ctx.recv, got, ctx.send)
    if ctx.static:
        rows = got.index_select(0, ctx.order.clamp_min(0))          # slot of each unique id
    else:
        rows = torch.empty_like(got)
        rows[ctx.order] = got
    return list(rows.split(dims, 1)) if len(tables) > 1 else [rows]


def _rows_apply_torch(table, sa, sb, rows, g, kind, lr, mu, nesterov, rho, eps, skip=None):
    """CPU twin of csrc/kernels/sparse_optim.hip (same per-row math)."""
    if skip is not None and int(skip.reshape(-1)[0]) != 0:
        return
    keep = rows >= 0
    r, gg = rows[keep], g[keep]
    var = table[r]
    if kind == 1:
        acc = mu * sa[r] + gg
        sa[r] = acc
        table[r] = var - lr * (gg + mu * acc if nesterov else acc)
    elif kind == 4:
        acc = sa[r] + gg * gg
        sa[r] = acc
        table[r] = var - lr * gg * torch.rsqrt(acc)
    elif kind == 5:
        ms = rho * sa[r] + (1 - rho) * gg * gg
        mom = mu * sb[r] + lr * gg * torch.rsqrt(ms + eps)
        sa[r], sb[r] = ms, mom
        table[r] = var - mom
    else:
        table[r] = var - lr * gg


def apply_sgd_shared(tables, ctx: LookupCtx, grads, lrs, grad_scale: float = 1.0):
    """The sparse update of every table (each table's `set_optimizer` rule,
    SGD by default); the gradients travel to the owners in ONE all-to-all
    (columns side by side, same routing as `lookup_shared`).  `grad_scale`
    multiplies the gradients (e.g. 1/W: the sync average) -- for SGD it is
    folded into the learning rate."""
    _check_shared(tables)
    t0 = tables[0]
    gs = [g.float().reshape(-1, t.dim) for t, g in zip(tables, grads)]
    if ctx.void is not None:       # a voided step: zero gradients make the scatter-SGD a no-op on every rank
        live = (1 - ctx.void).to(torch.float32)
        gs = [g * live for g in gs]
    if t0.W > 1:
        g = torch.cat(gs, 1) if len(gs) > 1 else gs[0]
        if ctx.static:
            # each live row has its own send slot (order = dest, unique), padding and
            # overflowed rows (-1) go to a dump row past the end: a plain scatter
            # copy (an atomic index_add_ of the [U, D] rows took 2.1 ms at B = 4096)
            n_send = sum(ctx.send)
            g_sorted = torch.zeros((n_send + 1, g.shape[1]), dtype=torch.float32, device=t0.device)
            dump = torch.full_like(ctx.order, n_send)
            g_sorted.index_copy_(0, torch.where(ctx.order >= 0, ctx.order, dump), g)
            g_sorted = g_sorted[:n_send]
        else:
            g_sorted = g[ctx.order].contiguous()
        recv_g = torch.empty((sum(ctx.recv), g.shape[1]), dtype=torch.float32, device=t0.device)
        t0.world.all_to_all(g_sorted, ctx.send, recv_g, ctx.recv)
        gs = list(recv_g.split([t.dim for t in tables], 1))
    for t, g, lr in zip(tables, gs, lrs):
        t._sgd_local(ctx, g.contiguous(), lr, grad_scale, ctx.void)


def _max_route_world() -> int:
    try:
        return ops._C().route_max_world()
    except Exception:       # CPU-only build without the extension: the torch emulation has no limit
        return 1 << 30


def _route_static_torch(sids: torch.Tensor, perm: torch.Tensor, W: int, cap: int):
    """CPU emulation of csrc/kernels/sparse_route.hip (same outputs)."""
    N = sids.numel()
    dev = sids.device
    flag = torch.ones(N, dtype=torch.bool, device=dev)
    flag[1:] = sids[1:] != sids[:-1]
    inv_sorted = (torch.cumsum(flag.to(torch.int64), 0) - 1).to(torch.int32)
    inverse = torch.empty(N, dtype=torch.int64, device=dev)
    inverse[perm] = inv_sorted.long()
    u = sids[flag].long()
    U = u.numel()
    uniq = torch.full((N,), -1, dtype=torch.int64, device=dev)
    uniq[:U] = u
    dest = torch.full((N,), -1, dtype=torch.int32, device=dev)
    send = torch.full((W * cap,), -1, dtype=torch.int64, device=dev)
    ocnt = torch.zeros(W, dtype=torch.int32, device=dev)
    if W > 1 and U:
        owner = u % W
        counts = torch.bincount(owner, minlength=W)
        ocnt = counts.to(torch.int32)
        start = torch.cumsum(counts, 0) - counts
        order = torch.argsort(owner, stable=True)          # id order within each owner
        pos = torch.empty(U, dtype=torch.int64, device=dev)
        pos[order] = torch.arange(U, device=dev) - start[owner[order]]
        fits = pos < cap                                    # an owner's ids beyond cap: not exchanged
        d = owner * cap + pos
        dest[:U] = torch.where(fits, d, torch.full_like(d, -1)).to(torch.int32)
        send[d[fits]] = u[fits]
    return inv_sorted, inverse, uniq, dest, send, ocnt


def pad_to_capacity(offsets: torch.Tensor, ids: torch.Tensor, vals: Optional[torch.Tensor], n_cap: int):
    """Pad a CSR batch's ids to the static capacity so captured steps see fixed
    shapes: the padding repeats the first id with weight 0 inside the LAST bag
    (a 'sum' combiner is unchanged, the dedup / owner counts too, and the
    gradient of a 0-weighted entry is 0).  Returns (offsets, ids, vals)."""
    n = ids.numel()
    if n > n_cap:
        raise ValueError(f"batch has {n} ids, above the static capacity {n_cap}")
    if vals is None:
        vals = torch.ones(n, dtype=torch.float32, device=ids.device)
    if n == n_cap:
        return offsets, ids, vals
    fill = ids[:1] if n > 0 else torch.zeros(1, dtype=ids.dtype, device=ids.device)
    ids = torch.cat([ids, fill.expand(n_cap - n)])
    vals = torch.cat([vals.float(), torch.zeros(n_cap - n, dtype=torch.float32, device=vals.device)])
    offsets = offsets.clone()
    offsets[-1] = n_cap
    return offsets, ids, vals


class StaticStepMixin:
    """The training-step driver shared by the sparse models (SparseLR, W&D):
    pads each batch to the static capacity, replays the captured graph when the
    shapes match (otherwise runs the same collectives eagerly: partial batches,
    CPU), and every `check_every` steps lets the router replay voided batches
    through the exact exchange and re-capture after a resize -- on every rank
    at the same step, so collective sequences always match.

    Needs: `_router()`, `_route_table()`, `_static_batch(batch)` (sets
    `_last_empty`), `_train_step(batch, exact)`, `_graphed`, `_example`,
    `_window`, `global_step`, `world`."""

    _last_empty = False

    def train_step(self, batch) -> torch.Tensor:
        b = self._static_batch(batch)
        empty = bool(self._last_empty)
        self._route_table().set_batch_empty(empty)
        g = self._graphed
        if g is not None and (g.matches(*b) or not g.strict):   # one rank: (re)capture lazily
            loss = g(*b)
        else:   # eager: the same collectives as the graph (partial batches, CPU, no graph)
            loss = self._train_step(b)
        self.global_step += 1
        r = self._router()
        if r is not None and self.world.world_size > 1:
            r.steps += 1
            self._window.append((b, empty))
            if r.due():
                self._check_exchange()
        return loss.detach()

    def sync_exchange(self):
        """Replay the voided steps of the current window now: afterwards every
        batch seen so far is applied.  Collective (every rank at the same
        point); evaluation, prediction, AUC and checkpoints call it first."""
        r = self._router()
        if r is not None and self.world.world_size > 1 and r.steps:
            self._check_exchange()

    def _check_exchange(self):
        r = self._router()
        voided, changed = r.check()
        window, self._window = self._window, []
        t = self._route_table()
        with torch.enable_grad():        # also reached from no_grad evaluation / prediction
            for i in voided:
                b, empty = window[i]
                t.set_batch_empty(empty)
                self._train_step(b, exact=True)
        t.set_batch_empty(False)
        if changed and self._graphed is not None and self._graphed.strict:
            self._graphed.capture(*self._example)
