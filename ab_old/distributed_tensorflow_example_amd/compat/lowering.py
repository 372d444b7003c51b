"""Graph lowering for Session.run: replace matched subgraphs by fused kernels.

The compat graph records TF op types and attrs on every node
(compat/graph.py), so a Session can recognise the reference's training
graph instead of running it op by op (Session.run -> fused step).
Matched today -- the headline graph (example.py:93-118):

    a2   = Sigmoid|Relu(Add|BiasAdd(MatMul(x, W1), b1))
    z3   = Add|BiasAdd(MatMul(a2, W2), b2)
    loss = Mean(Neg(Sum(Mul(y_, Log(Softmax(z3))), axis 1)))      naive form
         | Mean(SoftmaxCrossEntropyWithLogits(y_, z3))             stable form
    train_op = <Optimizer>.minimize(loss, global_step)
    accuracy = Mean(Cast(Equal(ArgMax(Softmax(z3), 1), ArgMax(y_, 1))))   (optional)

On one GPU with the MNIST loader's batches (uint8 source, one-hot labels) and
the reference's 784-100-10 shapes, a run that fetches train_op goes to the
RESIDENT engine (compat/resident.py): the persistent fp32 kernel
(csrc/kernels/mlp_persist_f32.hip) stays launched across runs and each run is
a pinned-memory doorbell -- no launch, no completion round trip.  Every other
case (float feeds, other shapes or optimizers, several workers) is the
launched plan: the exact-fp32 MFMA kernels of csrc/kernels/graph_mlp.hip
(forward + head + backward of layer 2 in one launch, the layer-1 weight
gradient in the second).  With GradientDescentOptimizer on one worker the
SGD update and global_step += 1 happen inside those kernels.  With N
synchronous workers on one node (example.py's ps/worker program as sync DP)
the kernels write this worker's gradients and ONE more kernel all-reduces
them with every worker's over the IPC data plane, in rank order, and applies
SGD + global_step on the graph's variables (csrc/bind_mlp.cpp
GraphStepPlan.attach_ipc, csrc/kernels/ipc_coll.hip reduce_sgd_k): no RCCL,
no host round trip, bit-identical replicas.  Other optimizers write the
gradients straight into the sync bucket (no copies) and the all-reduce +
fused optimizer step follow.  The loss and
accuracy of the run (pre-update, as TF evaluates them in the same run) are
seeded into the run's memo, so summaries / cost fetches of the same run cost
no extra kernels.

and lr2.py's sparse logistic regression (lr2.py:359-396) over a partitioned
(ps-placed, row-sharded) W:

    py_x = Add(EmbeddingLookupSparse(W, SparseTensor(idx, fids), SparseTensor(idx, fvals), 'sum'), b)
    loss = Mean(SigmoidCrossEntropyWithLogits(py_x, y))
    train_op = GradientDescentOptimizer(lr).minimize(loss, global_step)

whose train run becomes the native sparse-LR step on the variables' own
storage: on one GPU ONE native call (csrc/bind_sparse.cpp SparseLRPlan) packs
lr2.py's feed arrays (COO indices -> CSR offsets, int32 ids) into a pinned
slot with the GIL released, copies it once and runs the two kernels of
csrc/kernels/sparse_lr.hip (bag + sigmoid-xent, LDS-aggregated scatter SGD +
bias); with several workers, models/sparse_lr.py's sharded step (dedup,
routing, all-to-all) on packed feeds.

A run is lowered only if nothing else it fetches reads the matched
variables or interior nodes (those would see post-update weights); anything
unmatched -- other shapes, CPU tensors, other fetch sets -- runs eagerly as
before.  DTF_GRAPH_LOWERING=0 disables lowering.
"""
from __future__ import annotations

import os
import weakref
from typing import Any, Dict, List, Optional

import numpy as np
import torch

from .graph import Operation, Tensor

_CACHE: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()   # train_op -> plan | False


_MODS = {}


def _train_mod():
    """compat.train (imported lazily: it imports this module)."""
    m = _MODS.get("train")
    if m is None:
        from . import train as m
        _MODS["train"] = m
    return m


def _resident_mod():
    m = _MODS.get("resident")
    if m is None:
        from . import resident as m
        _MODS["resident"] = m
    return m


def _debug_mod():
    m = _MODS.get("debug")
    if m is None:
        from ..utils import debug as m
        _MODS["debug"] = m
    return m


def enabled() -> bool:
    return os.environ.get("DTF_GRAPH_LOWERING", "1") != "0"


def _is(t, *types) -> bool:
    return isinstance(t, Tensor) and getattr(t, "op_type", None) in types


def _is_plain_var(t) -> bool:
    return getattr(t, "op_type", None) == "VariableV2" and not getattr(t, "is_partitioned", False) and \
        isinstance(getattr(t, "value", None), torch.Tensor)


def _dense(t):
    """(lhs, W, b) of Add|BiasAdd(MatMul(lhs, W), b) with plain variables, else None."""
    if not _is(t, "Add", "AddV2", "BiasAdd") or len(t.inputs) != 2:
        return None
    mm, b = t.inputs
    if not _is(mm, "MatMul"):
        mm, b = b, mm
    if not _is(mm, "MatMul") or mm.attrs.get("transpose_a") or mm.attrs.get("transpose_b"):
        return None
    lhs, W = mm.inputs
    if not (_is_plain_var(W) and _is_plain_var(b)):
        return None
    if W.value.dim() != 2 or b.value.dim() != 1 or b.value.numel() != W.value.shape[1]:
        return None
    return lhs, W, b, [t, mm]


class MLPPattern:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def match_mlp(loss) -> Optional[MLPPattern]:
    """Match the reference loss graph; returns the pattern or None."""
    if not _is(loss, "Mean") or loss.attrs.get("axis") is not None:
        return None
    inner = loss.inputs[0]
    interior = [loss]
    naive = True
    if _is(inner, "SoftmaxCrossEntropyWithLogits"):
        if inner.attrs.get("dim", -1) not in (-1, 1):
            return None
        ylab, z3 = inner.inputs
        naive = False
        sm = None
        interior.append(inner)
    else:
        if not _is(inner, "Neg"):
            return None
        s = inner.inputs[0]
        if not _is(s, "Sum") or tuple(s.attrs.get("axis") or ()) not in ((1,), (-1,)) or s.attrs.get("keep_dims"):
            return None
        mul = s.inputs[0]
        if not _is(mul, "Mul") or len(mul.inputs) != 2:
            return None
        a, b = mul.inputs
        if not _is(b, "Log"):
            a, b = b, a
        if not _is(b, "Log"):
            return None
        sm = b.inputs[0]
        if not _is(sm, "Softmax") or sm.attrs.get("dim", -1) not in (-1, 1):
            return None
        ylab, z3 = a, sm.inputs[0]
        interior += [inner, s, mul, b, sm]
    d2 = _dense(z3)
    if d2 is None:
        return None
    a2, W2, b2, int2 = d2
    if not _is(a2, "Sigmoid", "Relu"):
        return None
    d1 = _dense(a2.inputs[0])
    if d1 is None:
        return None
    x, W1, b1, int1 = d1
    if W1.value.shape[1] != W2.value.shape[0]:
        return None
    if isinstance(ylab, Tensor) and (ylab is x):
        return None
    return MLPPattern(loss=loss, x=x, ylab=ylab, W1=W1, b1=b1, W2=W2, b2=b2, softmax=sm, z3=z3, a2=a2,
                      act=0 if a2.op_type == "Sigmoid" else 1, naive=naive,
                      interior=interior + int2 + [a2] + int1)


def _match_accuracy(g, pat) -> Optional[Tensor]:
    """Mean(Cast(Equal(ArgMax(y, 1), ArgMax(y_, 1)), float)) over the pattern's
    softmax (or logits) and labels, anywhere in the graph."""
    preds = {id(pat.z3)} | ({id(pat.softmax)} if pat.softmax is not None else set())
    for t in g._nodes:
        if not _is(t, "Mean") or t.attrs.get("axis") is not None:
            continue
        c = t.inputs[0]
        if not _is(c, "Cast") or c.attrs.get("DstT") not in (torch.float32,):
            continue
        e = c.inputs[0]
        if not _is(e, "Equal") or len(e.inputs) != 2:
            continue
        am = e.inputs
        if not all(_is(a, "ArgMax") and a.attrs.get("axis") in (1, -1) for a in am):
            continue
        srcs = [a.inputs[0] for a in am]
        for p, l in (srcs, srcs[::-1]):
            if (id(p) in preds or (_is(p, "Softmax") and p.inputs[0] is pat.z3)) and l is pat.ylab:
                return t
    return None


class _PlanBase:
    """fetches_ok: a lowered run is allowed only when no fetched node reads a
    matched variable or interior node (those would see post-update values)."""
    seeded: set
    blocked: set
    _fetch_ok: Dict[tuple, bool]

    def fetches_ok(self, fetch_list) -> bool:
        key = tuple(map(id, fetch_list))
        ok = self._fetch_ok.get(key)
        if ok is None:
            ok = True
            seen = set()
            stack = [f for f in fetch_list if isinstance(f, Tensor)]
            while stack and ok:
                t = stack.pop()
                if id(t) in seen or id(t) in self.seeded:
                    continue
                seen.add(id(t))
                if id(t) in self.blocked:
                    ok = False
                    break
                stack.extend(i for i in getattr(t, "inputs", ()) if isinstance(i, Tensor))
            self._fetch_ok[key] = ok
        return ok

    def fast_runner(self, flat):
        """A direct runner for this flat fetch list (Session._fast), or None."""
        return None


class MLPStepPlan(_PlanBase):
    """Fused execution of one matched train op."""

    def __init__(self, op: Operation, pat: MLPPattern, graph):
        info = op._lowering
        self.op, self.pat, self.info = op, pat, info
        self.accuracy = _match_accuracy(graph, pat)
        order = {id(v): i for i, v in enumerate(info["vars"])}
        self.var_index = [order[id(v)] for v in (pat.W1, pat.b1, pat.W2, pat.b2)]
        self.seeded = {id(pat.loss), id(op)} | ({id(self.accuracy)} if self.accuracy is not None else set())
        self.blocked = {id(t) for t in pat.interior} | {id(v) for v in (pat.W1, pat.b1, pat.W2, pat.b2)}
        self._fetch_ok: Dict[tuple, bool] = {}
        self.a2buf = self.dz2buf = self.metrics = None
        self.steps = 0
        self._rplan = None           # compat/resident.py handle (one worker, uint8 loader batches)
        self.resident_steps = 0

    # -------------------------------------------------------------- feeds
    @staticmethod
    def _feed_of(ctx, ph):
        if getattr(ph, "op_type", None) != "Placeholder" or id(ph) in ctx.memo:
            return None
        for key in (ph, ph.name, ph.name[:-2]):
            try:
                if key in ctx.feeds:
                    v = ctx.feeds[key]
                    return v if isinstance(v, np.ndarray) and v.dtype == np.float32 else None
            except TypeError:
                continue
        return None

    def _packed_feeds(self, ctx, dev):
        """x and y_ fed as float32 numpy arrays -> one pinned staging buffer ->
        ONE host-to-device copy (instead of one per placeholder)."""
        fx, fy = self._feed_of(ctx, self.pat.x), self._feed_of(ctx, self.pat.ylab)
        if fx is None or fy is None or fx.ndim != 2:
            return None
        nx, ny = fx.size, fy.size
        n = nx + ny
        slot = self._slot = (getattr(self, "_slot", 0) + 1) % 2
        if getattr(self, "_pinned", None) is None or self._pinned[0].numel() < n:
            cap = max(n, 1 << 16)
            self._pinned = [torch.empty(cap, dtype=torch.float32, pin_memory=True) for _ in range(2)]
            self._events = [None, None]
            self._dev = torch.empty(cap, dtype=torch.float32, device=dev)
        ev = self._events[slot]
        if ev is not None:
            ev.synchronize()                  # the copy that last read this staging slot is done
        hb = self._pinned[slot].numpy()
        hb[:nx] = fx.reshape(-1)
        hb[nx:n] = fy.reshape(-1)
        self._dev[:n].copy_(self._pinned[slot][:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._events[slot] = ev
        x = self._dev[:nx].view(fx.shape)
        y = self._dev[nx:n].view(fy.shape)
        ctx.memo[id(self.pat.x)] = x
        ctx.memo[id(self.pat.ylab)] = y
        return x, y

    # -------------------------------------------------------------- run
    def run(self, ctx, flat) -> bool:
        pat, info = self.pat, self.info
        W1, b1, W2, b2 = pat.W1.value, pat.b1.value, pat.W2.value, pat.b2.value
        if not W1.is_cuda:
            return False
        if self._run_native_plan(ctx, flat, W1, b1, W2, b2):
            return True
        from .. import _native
        _resident_mod().quiesce_all()   # the kernels below update the variables a resident engine holds
        xy = self._packed_feeds(ctx, W1.device)
        x, y = xy if xy is not None else (ctx.eval(pat.x), ctx.eval(pat.ylab))
        if not (isinstance(x, torch.Tensor) and isinstance(y, torch.Tensor) and x.is_cuda):
            return False
        if x.dtype != torch.float32 or y.dtype != torch.float32 or x.dim() != 2:
            return False
        B, K = x.shape
        H, C = W1.shape[1], W2.shape[1]
        HP, BP = (H + 16) // 16 * 16, (B + 15) // 16 * 16       # HP >= H + 1: the kernels' ones column
        if not (1 <= B <= 256 and BP * HP <= 16384 and H <= 128 and C <= 16 and W1.shape[0] == K
                and y.numel() == B * C and all(p.dtype == torch.float32 for p in (W1, b1, W2, b2))):
            return False
        x = x.contiguous()
        y = y.reshape(B, C).contiguous()
        if self.a2buf is None or self.a2buf.numel() < BP * HP:
            self.a2buf = torch.empty(BP * HP, dtype=torch.float32, device=x.device)
            self.dz2buf = torch.empty(BP * HP, dtype=torch.float32, device=x.device)
        if self.metrics is None:
            self.metrics = torch.zeros(3, dtype=torch.float32, device=x.device)
            self.host_metrics = torch.zeros(3, dtype=torch.float32, pin_memory=True)
        opt, fused, sync, gs_var = info["opt"], info["fused"], info["sync"], info["global_step"]
        _tr = _train_mod()
        GradientDescentOptimizer, _world_or_local = _tr.GradientDescentOptimizer, _tr._world_or_local
        _debug = _debug_mod()

        w = _world_or_local()
        opt._steps += 1
        _debug.fault_point(opt._steps, w.rank)
        lr = opt._lr_value()
        in_kernel = type(opt) is GradientDescentOptimizer and (w.world_size == 1 or not opt.sync_replicas) \
            and not info["sparse"]
        gstep = None
        if in_kernel and gs_var is not None and isinstance(getattr(gs_var, "value", None), torch.Tensor) \
                and gs_var.value.is_cuda and gs_var.value.numel() == 1 and \
                gs_var.value.dtype in (torch.float32, torch.int64, torch.int32, torch.float64):
            gstep = gs_var.value.data
        C_ = _native.load()
        if in_kernel:
            C_.graph_mlp_step(x, y, W1.data, b1.data, W2.data, b2.data, self.a2buf, self.dz2buf, None,
                              self.metrics, gstep, float(lr), pat.act, pat.naive, True)
            if gs_var is not None and gstep is None:
                with torch.no_grad():
                    gs_var.value.data += 1
        else:
            # gradients straight into the sync bucket's views (no copies), then one
            # synchronous update: the IPC all-reduce + SGD kernel for plain SGD,
            # else the all-reduce (IPC / RCCL) and the fused optimizer
            views = sync.views
            grads = [views[i] for i in self.var_index]
            C_.graph_mlp_step(x, y, W1.data, b1.data, W2.data, b2.data, self.a2buf, self.dz2buf, grads,
                              self.metrics, None, float(lr), pat.act, pat.naive, False)
            gl = [None] * len(info["vars"])
            for i, g in zip(self.var_index, grads):
                gl[i] = g
            done = sync.sgd(gl, lr, gs_var) if (type(opt) is GradientDescentOptimizer and opt.sync_replicas) \
                else None
            if done is None:
                if opt.sync_replicas:
                    gl = sync(gl)
                if fused is not None:
                    if isinstance(opt.learning_rate, Tensor):
                        fused.set_lr(lr)
                    fused.step(grads=[g.contiguous() for g in gl])
            if gs_var is not None and not done:
                with torch.no_grad():
                    gs_var.value.data += 1
        # loss / accuracy (/ global_step) of this run: one device-to-host copy
        # when the fetches need them, seeded as host scalars
        needs, gs_seed, _ = self._needs(flat, gs_var, gstep)
        if needs:
            self.host_metrics.copy_(self.metrics)
            m = self.host_metrics
            ctx.memo[id(pat.loss)] = m[0]
            if self.accuracy is not None:
                ctx.memo[id(self.accuracy)] = m[1]
            if gs_seed:
                ctx.memo[id(gs_var)] = m[2].to(gs_var.value.dtype)
        else:
            ctx.memo[id(pat.loss)] = self.metrics[0]
            if self.accuracy is not None:
                ctx.memo[id(self.accuracy)] = self.metrics[1]
        ctx.memo[id(self.op)] = None
        self.steps += 1
        return True

    def _run_native_plan(self, ctx, flat, W1, b1, W2, b2) -> bool:
        """The reference's case -- plain SGD (one worker, or async), numpy feeds --
        as ONE native call: C++ packs the feeds (GIL released), one host-to-device
        copy, the three kernels; the last kernel stores loss / accuracy /
        global_step into pinned host memory (csrc/bind_mlp.cpp GraphStepPlan).
        The checks that need tensor attribute calls (dtype, contiguity, data
        pointers: ~1 us each from Python) run only when the variables' value
        objects or the feed shapes change; the fetched values are seeded as numpy
        scalars read from the pinned buffer (no tensor indexing / .cpu() per
        fetch).  False: not applicable."""
        _tr = _train_mod()
        GradientDescentOptimizer, _world_or_local = _tr.GradientDescentOptimizer, _tr._world_or_local
        _debug = _debug_mod()

        pat, info = self.pat, self.info
        opt, gs_var = info["opt"], info["global_step"]
        w = _world_or_local()
        if type(opt) is not GradientDescentOptimizer or info["sparse"]:
            return False
        if w.world_size > 1 and opt.sync_replicas and self._sync_ipc(w) is None:
            return False       # several synchronous workers: only over the IPC data plane
        fx, fy = self._feed_of(ctx, pat.x), self._feed_of(ctx, pat.ylab)
        if fx is None or fy is None or fx.ndim != 2:
            return False
        gv = getattr(gs_var, "value", None) if gs_var is not None else None
        fast = (id(W1), id(b1), id(W2), id(b2), id(gv), fx.shape, fy.size)
        if getattr(self, "_fast_key", None) != fast:
            if not self._build_native_plan(fx, fy, W1, b1, W2, b2, gs_var, gv, w):
                self._fast_key = None
                return False
            self._fast_key = fast
        B, C = self._cplan_BC
        opt._steps += 1
        _debug.fault_point(opt._steps, w.rank)
        needs, gs_seed, scalars = self._needs(flat, gs_var, self._gstep)
        fy2 = (fy if fy.flags.c_contiguous else np.ascontiguousarray(fy)).reshape(B, C)
        u8 = getattr(fx, "u8", None)
        u8_ok = (u8 is not None and self._cplan_u8 and not fx.flags.writeable and u8.shape == fx.shape
                 and u8.dtype == np.uint8 and fx.shape[1] % 4 == 0)
        res = _resident_mod()
        if u8_ok and self._rplan is not None and self._rplan.run_u8(u8, fy2, float(opt._lr_value())):
            # the resident engine (compat/resident.py): no launch / completion per run
            ctx.resident_ran = True
            m = self._rplan.out if scalars else torch.from_numpy(self._rplan.out.copy())
            memo = ctx.memo
            memo[id(pat.loss)] = m[0]
            if self.accuracy is not None:
                memo[id(self.accuracy)] = m[1]
            if gs_seed:
                memo[id(gs_var)] = self._rplan.out[2]
            memo[id(self.op)] = None
            self.steps += 1
            self.resident_steps = getattr(self, "resident_steps", 0) + 1
            return True
        if res.any_live():
            res.quiesce_all()           # the launched plans below write the same variables
        if u8_ok:
            # data/mnist.py PixelBatch: ship the uint8 source (bit-identical, 4x fewer bytes)
            self._cplan.run_u8(u8, fy2, float(opt._lr_value()), bool(needs))
        else:
            self._cplan.run(fx if fx.flags.c_contiguous else np.ascontiguousarray(fx), fy2,
                            float(opt._lr_value()), bool(needs))
        # pinned host metrics [loss, accuracy, global_step]: numpy view -> float32
        # scalar copies, or 0-d tensors when another node of the run consumes them
        m = self._hm_np if scalars else self._cplan.host_metrics().clone()
        memo = ctx.memo
        memo[id(pat.loss)] = m[0]          # numpy float32 scalars (copies)
        if self.accuracy is not None:
            memo[id(self.accuracy)] = m[1]
        if gs_seed:
            memo[id(gs_var)] = self._hm_np[2]   # float32 global_step (gs_seed requires it)
        memo[id(self.op)] = None
        self.steps += 1
        return True

    def _sync_ipc(self, w):
        """The IpcColl the native plan's synchronous step reduces over, or None.
        COLLECTIVE on the first call (every worker's first lowered run): the
        node's IPC data plane comes up (or is refused) on all ranks alike."""
        if not hasattr(self, "_ipc"):
            coll = w.gpu_coll(4 * sum(v.value.numel() for v in self.info["vars"]))
            self._ipc = coll if (coll is not None and coll is w.ipc and self.info["sync"] is not None
                                 and self.info["sync"].comm_dtype in (None, torch.float32)) else None
        return self._ipc

    def _build_native_plan(self, fx, fy, W1, b1, W2, b2, gs_var, gv, w=None) -> bool:
        from .. import _native

        pat = self.pat
        B, K = fx.shape
        H, C = W1.shape[1], W2.shape[1]
        HP, BP = (H + 16) // 16 * 16, (B + 15) // 16 * 16
        if not (1 <= B <= 256 and BP * HP <= 16384 and H <= 128 and C <= 16 and W1.shape[0] == K
                and fy.size == B * C and all(p.dtype == torch.float32 and p.is_contiguous()
                                             for p in (W1, b1, W2, b2))):
            return False
        gstep = None
        if gs_var is not None:
            if not (isinstance(gv, torch.Tensor) and gv.is_cuda and gv.numel() == 1
                    and gv.dtype in (torch.float32, torch.int64, torch.int32, torch.float64)):
                return False
            gstep = gv.data
        key = (B, K, W1.data_ptr(), b1.data_ptr(), W2.data_ptr(), b2.data_ptr(),
               None if gstep is None else gstep.data_ptr(), pat.act, pat.naive)
        if getattr(self, "_cplan_key", None) != key:
            multi = w is not None and w.world_size > 1 and self.info["opt"].sync_replicas
            # direct launches by default (measured: a hipGraph replay's fixed host cost
            # exceeds three direct launches here); DTF_GRAPH_STEP_HIPGRAPH=1 replays one
            # (one worker only)
            self._cplan = _native.load().GraphStepPlan(W1.data, b1.data, W2.data, b2.data, gstep, B, pat.act,
                                                       bool(pat.naive),
                                                       os.environ.get("DTF_GRAPH_STEP_HIPGRAPH", "0") == "1"
                                                       and not multi)
            self._cplan_key = key
            if multi:
                # several workers: the plan's step ends with the IPC all-reduce + SGD kernel
                self._cplan.attach_ipc(self._sync_ipc(w))
            self._hm_np = self._cplan.host_metrics().numpy()
            # the captured-graph plan takes float32 feeds only (run_u8 is direct-launch)
            self._cplan_u8 = not self._cplan.use_graph()
            # the resident engine: one worker, the reference's shapes, uint8 loader batches
            # (compat/resident.py; the persistent kernel takes batches <= its max)
            old = getattr(self, "_rplan", None)
            if old is not None:
                old.stop()
            self._rplan = None
            res = _resident_mod()
            C_ = _native.load()
            if (res.enabled() and self._cplan_u8 and (w is None or w.world_size == 1) and K == 784 and H == 100
                    and C == 10 and B <= C_.mlpf_max_batch()):
                self._rplan = res.ResidentHandle(C_.ResidentMLPPlan(
                    W1.data, b1.data, W2.data, b2.data, gstep, B, pat.act, bool(pat.naive), res.idle_s()))
        self._cplan_BC = (B, C)
        self._gstep = gstep
        return True

    def fast_runner(self, flat):
        """The resident engine's run without the Session's per-run machinery
        (Session._fast): once a run of exactly these fetches went to the resident
        engine, the next runs hand the loader's uint8 batch and the labels from
        the feed dict (keyed by the placeholders themselves) straight to
        ResidentMLPPlan.run_u8 and read the fetched scalars from its pinned
        metrics.  Taken only when nothing per-run can differ: a constant learning
        rate, no fault injection, fetches among {train op, loss, accuracy,
        global_step} with global_step seeded by the engine.  Any other feed
        returns None and the run takes the full path."""
        rp = getattr(self, "_rplan", None)
        if rp is None or getattr(self, "_fast_key", None) is None:
            return None
        opt, gs_var = self.info["opt"], self.info["global_step"]
        if isinstance(opt.learning_rate, Tensor) or os.environ.get("DTF_FAULT_STEP") is not None:
            return None
        pat, acc = self.pat, self.accuracy
        kinds = []
        for f in flat:
            if f is self.op:
                kinds.append(-1)
            elif f is pat.loss:
                kinds.append(0)
            elif acc is not None and f is acc:
                kinds.append(1)
            elif gs_var is not None and f is gs_var:
                kinds.append(2)
            else:
                return None
        needs, gs_seed, scalars = self._needs(flat, gs_var, self._gstep)
        if not scalars or (2 in kinds and not gs_seed):
            return None
        lr = float(opt.learning_rate)
        B, C = self._cplan_BC
        xph, yph, nd = pat.x, pat.ylab, np.ndarray
        self.resident_steps = getattr(self, "resident_steps", 0)
        shape = (B, 784)

        prun, out, u8t, f32t, n = rp.plan.run_u8, rp.out, np.dtype(np.uint8), np.dtype(np.float32), B * C
        live = _resident_mod()._LIVE

        def fast(feed):
            # this runner belongs to ONE resident handle: once the plan was rebuilt
            # (another batch shape stopped `rp` and made a new engine) or any other
            # engine is live, take the full path -- relaunching `rp` next to a live
            # engine would train the same variables from two register copies
            if self._rplan is not rp or (live and (len(live) > 1 or live[0] is not rp)):
                return None
            fx, fy = feed.get(xph), feed.get(yph)
            u8 = getattr(fx, "u8", None)
            if (u8 is None or not isinstance(fx, nd) or fx.flags.writeable or fx.shape != shape
                    or type(u8) is not nd or u8.dtype != u8t or u8.shape != shape
                    or type(fy) is not nd or fy.dtype != f32t or fy.size != n or not fy.flags.c_contiguous):
                return None
            # (a run that registers the engine as live goes through the handle)
            if not (prun(u8, fy, lr) if rp.live else rp.run_u8(u8, fy, lr)):
                return None
            opt._steps += 1
            self.steps += 1
            self.resident_steps += 1
            return [None if k < 0 else out[k] for k in kinds]
        fast.stale = lambda: self._rplan is not rp       # try_lower replaces a stale runner
        return fast

    def _needs(self, flat, gs_var, gstep):
        """(fetches read the loss/accuracy, global_step may be seeded)."""
        key = ("needs",) + tuple(map(id, flat))
        r = self._fetch_ok.get(key)
        if r is None:
            targets = {id(self.pat.loss)} | ({id(self.accuracy)} if self.accuracy is not None else set())
            hit, seen = False, {}
            stack = [f for f in flat if isinstance(f, Tensor) and f is not self.op]
            while stack:
                t = stack.pop()
                if id(t) in seen:
                    continue
                seen[id(t)] = t
                if id(t) in targets:
                    hit = True
                    continue
                stack.extend(i for i in getattr(t, "inputs", ()) if isinstance(i, Tensor))
            # global_step is seeded (post-increment, exact in fp32) only when it is
            # fetched directly and no other node of the run reads it
            def read_by_others(v):
                return any(i is v for t in seen.values() for i in getattr(t, "inputs", ()))
            gs_ok = (gstep is not None and gstep.dtype == torch.float32 and any(f is gs_var for f in flat)
                     and not read_by_others(gs_var))
            # loss / accuracy may be seeded as numpy scalars when only fetched directly
            # (a consuming node -- a summary, a reduction -- gets a tensor)
            scalars = not read_by_others(self.pat.loss) and (self.accuracy is None
                                                               or not read_by_others(self.accuracy))
            r = (hit or gs_ok, gs_ok, scalars)
            self._fetch_ok[key] = r
        return r

class SparseLRPattern:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def _placeholder(t) -> bool:
    return getattr(t, "op_type", None) == "Placeholder"


def match_sparse_lr(loss) -> Optional[SparseLRPattern]:
    """lr2.py:383-391 -- mean sigmoid xent of (sum-combined sparse lookup of a
    partitioned [F, 1] W) + b, every input a placeholder."""
    if not _is(loss, "Mean") or loss.attrs.get("axis") is not None or not loss.inputs:
        return None
    xent = loss.inputs[0]
    if not _is(xent, "SigmoidCrossEntropyWithLogits") or len(xent.inputs) != 2:
        return None
    logits, y = xent.inputs
    if not _is(logits, "Add", "AddV2", "BiasAdd") or len(logits.inputs) != 2:
        return None
    e, b = logits.inputs
    if not _is(e, "EmbeddingLookupSparse"):
        e, b = b, e
    if not _is(e, "EmbeddingLookupSparse") or e.attrs.get("combiner") != "sum" or len(e.inputs) != 2:
        return None
    W = getattr(e, "params", None)
    if not (getattr(W, "is_partitioned", False) and getattr(W, "dim", 0) == 1):
        return None
    if not (_is_plain_var(b) and b.value.numel() == 1 and b.value.dtype == torch.float32):
        return None
    sp_ids, sp_w = e.inputs
    if sp_w is None or getattr(sp_ids, "indices", None) is None or getattr(sp_w, "indices", None) is not sp_ids.indices:
        return None
    idx, fids, fvals = sp_ids.indices, sp_ids.values, sp_w.values
    if not all(_placeholder(t) for t in (idx, fids, fvals, y)):
        return None
    return SparseLRPattern(loss=loss, W=W, b=b, y=y, idx=idx, fids=fids, fvals=fvals,
                           interior=[loss, xent, logits, e, sp_ids, sp_w])


class SparseLRStepPlan(_PlanBase):
    """lr2.py's train run on the native sparse-LR step over the graph's own
    variables (W's shards, b's tensor): same synchronous semantics as the
    op-by-op path (sum of the per-worker mean gradients / W, owner-side scatter
    SGD), one host-to-device copy of the packed feeds, and on one GPU a
    hipGraph replay per (batch rows, padded id count)."""

    ID_BUCKET = 4096       # ids padded to a multiple of this (a handful of captured shapes)

    def __init__(self, op: Operation, pat: SparseLRPattern):
        self.op, self.pat, self.info = op, pat, op._lowering
        self.seeded = {id(pat.loss), id(op)}
        self.blocked = {id(t) for t in pat.interior} | {id(pat.W), id(pat.b)}
        self._fetch_ok = {}
        self.trainer = None
        self._stage = None
        self._nplan = None            # one worker: csrc/bind_sparse.cpp SparseLRPlan
        self._fused_env = os.environ.get("DTF_SLR_FUSED", "1") != "0"
        # the one-GPU kernels skip (and count) feature ids outside [0, F); TF's
        # gather raises InvalidArgument.  The count is read back every
        # DTF_SPARSE_ID_CHECK runs (0: never) and a nonzero count raises here.
        self._id_check = int(os.environ.get("DTF_SPARSE_ID_CHECK", "256"))
        self.steps = 0

    @staticmethod
    def _feed(ctx, ph):
        for key in (ph, ph.name, ph.name[:-2]):
            try:
                if key in ctx.feeds:
                    return ctx.feeds[key]
            except TypeError:
                continue
        return None

    def _batch(self, ctx, dev):
        """(labels [B,1], offsets [B+1], ids, vals) on `dev` from the feeds, or
        None (then the run goes op by op)."""
        p = self.pat
        fy, fi, ff, fv = (self._feed(ctx, t) for t in (p.y, p.idx, p.fids, p.fvals))
        if any(v is None or isinstance(v, torch.Tensor) for v in (fy, fi, ff, fv)):
            return None
        y = np.asarray(fy, dtype=np.float32)
        idx = np.asarray(fi)
        ids = np.asarray(ff).astype(np.int64, copy=False).reshape(-1)
        vals = np.asarray(fv, dtype=np.float32).reshape(-1)
        B = y.shape[0] if y.ndim else 0
        nnz = ids.size
        if B == 0 or y.size != B or vals.size != nnz or (nnz and (idx.ndim != 2 or idx.shape[0] != nnz)):
            return None
        rows = idx[:, 0] if nnz else np.zeros(0, np.int64)
        if nnz and (rows.min() < 0 or rows.max() >= B):
            return None
        if nnz and (rows[1:] < rows[:-1]).any():
            # not in canonical row order: a stable sort by row gives the same bags
            # (sum combiner), so every rank lowers -- the decision must not depend on
            # one rank's data (ranks that lowered and ranks that went op by op would
            # issue different collectives)
            order = np.argsort(rows, kind="stable")
            rows, ids, vals = rows[order], ids[order], vals[order]
        offsets = np.zeros(B + 1, np.int64)
        if nnz:
            np.cumsum(np.bincount(rows, minlength=B), out=offsets[1:])
        pad = 0
        if dev.type == "cuda" and self.trainer is not None and self.trainer.world.world_size == 1 and nnz:
            pad = -(-nnz // self.ID_BUCKET) * self.ID_BUCKET - nnz
        n = nnz + pad
        if dev.type != "cuda":
            to = lambda a: torch.from_numpy(np.ascontiguousarray(a))
            lab, off, i, v = to(y.reshape(B, 1)), to(offsets), to(ids), to(vals)
        else:
            # one pinned staging buffer -> one copy: [ids i64 | offsets i64 | vals f32 | labels f32]
            sizes = [8 * n, 8 * (B + 1), 4 * n, 4 * B]
            offs = np.cumsum([0] + [-(-s // 16) * 16 for s in sizes])
            total = int(offs[-1])
            if self._stage is None or self._stage[0].numel() < total:
                cap = max(total, 1 << 20)
                self._stage = [torch.empty(cap, dtype=torch.uint8, pin_memory=True),
                               torch.empty(cap, dtype=torch.uint8, device=dev), None]
            host, devb, ev = self._stage
            if ev is not None:
                ev.synchronize()                   # the previous copy out of the staging buffer is done
            hb = host.numpy()
            hv = [hb[offs[k]:offs[k] + sizes[k]] for k in range(4)]
            hi = hv[0].view(np.int64)
            hi[:nnz] = ids
            hi[nnz:] = ids[0] if nnz else 0        # padding repeats the first id with weight 0 (last bag)
            hv[1].view(np.int64)[:] = offsets
            if pad:
                hv[1].view(np.int64)[-1] = n
            hf = hv[2].view(np.float32)
            hf[:nnz] = vals
            hf[nnz:] = 0.0
            hv[3].view(np.float32)[:] = y.reshape(-1)
            devb[:total].copy_(host[:total], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._stage[2] = ev
            dv = [devb[int(offs[k]):int(offs[k]) + sizes[k]] for k in range(4)]
            i, off = dv[0].view(torch.int64), dv[1].view(torch.int64)
            v, lab = dv[2].view(torch.float32), dv[3].view(torch.float32).view(B, 1)
        return lab, off, i, v

    def _native_run(self, ctx, opt, gs_var, table) -> bool:
        """One worker: the whole run as ONE native call on lr2.py's own feed
        arrays (csrc/bind_sparse.cpp SparseLRPlan: CSR build + packing with the
        GIL released, one copy, two kernels -- no dedup or routing needed when
        every row of W is local).  False: feeds it does not take (tensors, other
        dtypes, a row outside the batch)."""
        p = self.pat
        fy, fi, ff, fv = (self._feed(ctx, t) for t in (p.y, p.idx, p.fids, p.fvals))
        if not all(isinstance(v, np.ndarray) for v in (fy, fi, ff, fv)):
            return False
        if self._nplan is None:
            from .. import _native

            gv = getattr(gs_var, "value", None) if gs_var is not None else None
            gst = gv.data if (isinstance(gv, torch.Tensor) and gv.is_cuda and gv.numel() == 1 and gv.dtype in (
                torch.float32, torch.int64, torch.int32, torch.float64)) else None
            self._nplan = _native.load().SparseLRPlan(table.local, p.b.value.data, gst)
            self._nplan_gs = gst is not None
        if not self._nplan.run(fy, fi, ff, fv, float(opt._lr_value())):
            return False
        opt._steps += 1
        if self._id_check and opt._steps % self._id_check == 0:
            self.check_ids()
        _debug_mod().fault_point(opt._steps, 0)
        if gs_var is not None and not self._nplan_gs:
            with torch.no_grad():
                gs_var.value.data += 1
        ctx.memo[id(p.loss)] = self._nplan.loss()   # this run's loss (a device scalar, read before the next run)
        ctx.memo[id(self.op)] = None
        self.steps += 1
        return True

    def check_ids(self):
        """Raise InvalidArgumentError (ValueError) if any run since the plan was
        built fed a feature id outside [0, F) (those ids were skipped: their bags
        trained truncated, where TF's embedding gather would have failed the run)."""
        if self._nplan is None:
            return
        n = int(self._nplan.bad_ids())
        if n:
            raise ValueError(f"embedding_lookup_sparse: {n} feature id(s) outside [0, {self.pat.W.table.num_rows}) "
                             f"were fed to the sparse-LR step (skipped on the device; TF raises "
                             f"InvalidArgument)")

    def fast_runner(self, flat):
        """The one-GPU native step without the Session's per-run machinery: once a
        run of exactly these fetches went through _native_run, the next runs call
        SparseLRPlan.run on the four feeds straight from the feed dict (keyed by
        the placeholders themselves).  Taken only when nothing per-run can differ:
        a constant learning rate, global_step advanced on the device, no fault
        injection; the fetches are the train op and / or the loss.  Any other
        feed shape returns None and the run takes the full path."""
        if self._nplan is None or (self.info["global_step"] is not None and not self._nplan_gs):
            return None
        opt = self.info["opt"]
        if isinstance(opt.learning_rate, Tensor) or os.environ.get("DTF_FAULT_STEP") is not None:
            return None
        if not all(f is self.op or f is self.pat.loss for f in flat):
            return None
        lr = float(opt.learning_rate)
        p, nplan, res = self.pat, self._nplan, _resident_mod()
        y, idx, fids, fvals = p.y, p.idx, p.fids, p.fvals
        want_loss = [f is p.loss for f in flat]
        nd, check = np.ndarray, self._id_check

        def fast(feed):
            fy, fi, ff, fv = feed.get(y), feed.get(idx), feed.get(fids), feed.get(fvals)
            if type(fy) is not nd or type(fi) is not nd or type(ff) is not nd or type(fv) is not nd or res._LIVE:
                return None
            if not nplan.run(fy, fi, ff, fv, lr):
                return None
            opt._steps += 1
            self.steps += 1
            if check and opt._steps % check == 0:
                self.check_ids()
            return [nplan.loss().cpu().numpy() if wl else None for wl in want_loss]
        return fast

    def run(self, ctx, flat) -> bool:
        from ..models.sparse_lr import SparseLRTrainer
        _debug = _debug_mod()
        _tr = _train_mod()
        GradientDescentOptimizer, _world_or_local = _tr.GradientDescentOptimizer, _tr._world_or_local

        p, info = self.pat, self.info
        opt, gs_var = info["opt"], info["global_step"]
        w = _world_or_local()
        if type(opt) is not GradientDescentOptimizer or (w.world_size > 1 and not opt.sync_replicas):
            return False
        _resident_mod().quiesce_all()
        table = p.W.table
        if table.hogwild is not None:
            return False
        dev = table.device
        if dev.type == "cuda" and w.world_size == 1 and self._fused_env and self._native_run(ctx, opt, gs_var, table):
            return True
        if self.trainer is None:
            self.trainer = SparseLRTrainer(table.num_rows, float(opt._lr_value()), w, device=dev, table=table,
                                           bias=p.b.value)
            if dev.type == "cuda" and w.world_size == 1:
                self.trainer.enable_graph()        # one worker: no collectives, lazy per-shape captures
        if any(v is None or isinstance(v, torch.Tensor)
               for v in (self._feed(ctx, t) for t in (p.y, p.idx, p.fids, p.fvals))):
            # feed KINDS are the same on every rank (the graph's placeholders fed the
            # same way): every rank goes op by op together
            return False
        batch = self._batch(ctx, dev)
        if batch is None:
            if w.world_size > 1:
                # falling back on this rank alone would desynchronise the collectives
                # of the lowered step (all-to-all / all-reduce) from its peers'
                raise RuntimeError("lowered sparse-LR step: this worker's feeds do not match the graph (label / "
                                   "index size mismatch or out-of-range rows); synchronous workers "
                                   "cannot fall back op by op one rank at a time")
            return False
        opt._steps += 1
        _debug.fault_point(opt._steps, w.rank)
        self.trainer.lr = float(opt._lr_value())
        loss = self.trainer.train_step(batch)
        if gs_var is not None:
            with torch.no_grad():
                gs_var.value.data += 1
        ctx.memo[id(p.loss)] = loss.clone()        # pre-update loss of this run (a graph's output is reused)
        ctx.memo[id(self.op)] = None
        self.steps += 1
        return True


def _flatten(f, out: List[Any]):
    if isinstance(f, (list, tuple)):
        for x in f:
            _flatten(x, out)
    elif isinstance(f, dict):
        for x in f.values():
            _flatten(x, out)
    elif f is not None:
        out.append(f)
    return out


def try_lower(session, fetches, ctx, flat=None) -> None:
    """Run lowered plans for train ops in `fetches`, seeding ctx.memo."""
    lower = getattr(session, "_lower", None)          # read once per Session (compat/session.py)
    if not (enabled() if lower is None else lower):
        return
    if flat is None:
        flat = _flatten(fetches, [])
    for f in flat:
        if getattr(f, "_lowering", None) is None or not isinstance(f, Operation):
            continue
        plan = f.__dict__.get("_dtf_plan")
        if plan is None:
            plan = _CACHE.get(f)
        if plan is None:
            loss = getattr(f, "loss", None)
            pat = match_mlp(loss) if loss is not None else None
            plan = False
            if pat is not None and pat.W1.value.is_cuda and {id(v) for v in f._lowering["vars"]} == \
                    {id(v) for v in (pat.W1, pat.b1, pat.W2, pat.b2)}:
                plan = MLPStepPlan(f, pat, session.graph)     # (GPU kernels: CPU sessions run it op by op)
            elif loss is not None:
                sp = match_sparse_lr(loss)
                if sp is not None and [id(v) for v in f._lowering["vars"]] == [id(sp.b)] and \
                        [id(pv) for _, pv in f._lowering["sparse"]] == [id(sp.W)]:
                    plan = SparseLRStepPlan(f, sp)
            _CACHE[f] = plan
            f._dtf_plan = plan
        if plan is False or id(f) in ctx.memo:
            continue
        if plan.fetches_ok(flat) and plan.run(ctx, flat) and flat is fetches and \
                isinstance(getattr(session, "_fast", None), dict):
            fk = tuple(map(id, flat))
            old = session._fast.get(fk)
            if old is None or (getattr(old, "stale", None) is not None and old.stale()):
                session._fast.pop(fk, None)
                runner = plan.fast_runner(flat)
                if runner is not None:
                    session._fast[fk] = runner


def plan_for(train_op) -> Optional[_PlanBase]:
    p = _CACHE.get(train_op)
    return p if p else None
