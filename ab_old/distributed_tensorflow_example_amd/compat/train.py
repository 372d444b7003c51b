"""tf.train equivalents: Server, replica_device_setter, optimizers,
SyncReplicasOptimizer, Supervisor, MonitoredTrainingSession + hooks, Saver.

Semantics shift: the reference trains asynchronously
against one parameter server (between-graph replication, Hogwild updates).
Here every worker holds a full replica on its own GPU and each `train_op`
run is one *synchronous* data-parallel step: local gradients are averaged by
an all-reduce (RCCL over xGMI on GPU, gloo on CPU) and applied by the fused
optimizer kernel.  `global_step` therefore counts synchronous steps (not
worker-steps).  Chief-only init + broadcast replaces every worker re-running
init_op (the lr2.py:419 race, A6); ps tasks are control-plane members that
exit when all workers have sent their done token (lr2.py:337-346 intent).
"""
from __future__ import annotations

import atexit
import contextlib
import os
import threading
import time
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import optim as _optim
from ..utils import debug as _debug
from ..utils import profiling as _prof
from ..parallel import async_ps as _async_ps
from ..parallel import world as _world
from ..parallel.cluster import ClusterSpec, Rendezvous, split_address
from ..utils import logging as _log
from . import saver as _saver
from .graph import (GLOBAL_STEP, GLOBAL_VARIABLES, LOCAL_VARIABLES, TRAINABLE_VARIABLES, Operation,
                    RunContext, Tensor, Variable, constant_initializer, get_default_graph, get_variable,
                    global_variables, local_variables, trainable_variables)
from .queues import (Coordinator, QueueRunner, add_queue_runner, batch, shuffle_batch, slice_input_producer,
                     start_queue_runners, string_input_producer)
from .saver import (CheckpointReader, NewCheckpointReader, Saver, checkpoint_exists, export_meta_graph,
                    get_checkpoint_state, latest_checkpoint, list_variables, load_variable, read_meta_graph,
                    update_checkpoint_state)
from .session import ConfigProto, Session
from .summary import FileWriter, SummaryWriter

__all__ = [
    "ClusterSpec", "Server", "replica_device_setter", "GradientDescentOptimizer", "MomentumOptimizer",
    "AdamOptimizer", "AdagradOptimizer", "RMSPropOptimizer", "SyncReplicasOptimizer", "Supervisor",
    "MonitoredTrainingSession", "MonitoredSession", "SingularMonitoredSession", "Scaffold", "Saver",
    "export_meta_graph", "read_meta_graph",
    "Coordinator", "QueueRunner", "start_queue_runners", "add_queue_runner", "batch", "shuffle_batch",
    "slice_input_producer", "string_input_producer", "latest_checkpoint", "get_checkpoint_state",
    "get_global_step", "get_or_create_global_step", "create_global_step", "global_step", "SummaryWriter",
    "SessionRunHook", "SessionRunArgs", "StopAtStepHook", "CheckpointSaverHook", "SummarySaverHook",
    "LoggingTensorHook", "NanTensorHook", "StepCounterHook", "FinalOpsHook", "NanLossDuringTrainingError",
]

_SERVER: Optional["Server"] = None


# ======================================================================= Server
class Server:
    """tf.train.Server: one per task.  Joins the cluster rendezvous (native TCP
    store hosted by worker:0) and, for workers, the data-parallel world."""

    def __init__(self, server_or_cluster_def, job_name: str = None, task_index: int = 0, protocol=None,
                 config=None, start: bool = True, timeout_s: float = None):
        global _SERVER
        cluster = server_or_cluster_def
        if isinstance(cluster, dict):
            cluster = ClusterSpec(cluster)
        if not isinstance(cluster, ClusterSpec):
            raise TypeError("Server needs a ClusterSpec or dict")
        if not job_name:
            raise ValueError("job_name is required (e.g. --job_name=worker)")
        self.cluster = cluster
        self.job_name = job_name
        self.task_index = int(task_index)
        self.server_def = {"cluster": cluster.as_dict(), "job_name": job_name, "task_index": self.task_index}
        timeout_s = float(timeout_s or os.environ.get("DTF_RENDEZVOUS_TIMEOUT", 300))
        self.rdv = Rendezvous(cluster, job_name, self.task_index, timeout_s=timeout_s)
        host, port = split_address(cluster.task_address(job_name, self.task_index))
        self.target = f"dtf://{host}:{port}"
        self.world = None
        if self.rdv.is_worker:
            backend = os.environ.get("DTF_BACKEND", "auto")
            self.world = _world.init_from_rendezvous(self.rdv, backend=backend, timeout_s=timeout_s)
            get_default_graph().device = self.world.device
        self.rdv.start_heartbeat()
        self._done = False
        self._start_watchdog()
        _SERVER = self
        atexit.register(self._atexit)

    @property
    def is_chief(self) -> bool:
        return self.rdv.is_chief

    def _start_watchdog(self):
        """Failure detection: a worker whose peer stopped heart-beating aborts its
        RCCL communicator and exits non-zero instead of blocking forever in a
        collective (the launcher then tears the job down; restart resumes from
        the last checkpoint).  DTF_PEER_TIMEOUT seconds (0 disables)."""
        stale = float(os.environ.get("DTF_PEER_TIMEOUT", "60"))
        if stale <= 0 or not self.rdv.is_worker or self.rdv.num_workers < 2:
            return

        def watch():
            while not self._done:
                time.sleep(min(2.0, stale / 4))
                try:
                    dead = [d for d in self.rdv.dead_workers(stale_s=stale) if d != self.task_index]
                except Exception:  # noqa: BLE001 - store gone: chief exited
                    return
                if dead and not self._done:
                    _log.error(f"[{self.job_name}:{self.task_index}] workers {dead} stopped responding; aborting")
                    try:
                        if self.world is not None and self.world.comm is not None:
                            self.world.comm.abort()
                    finally:
                        os._exit(3)
        threading.Thread(target=watch, daemon=True, name="dtf-watchdog").start()

    def start(self):
        return self

    def join(self, timeout: float = -1.0):
        """ps: block until every worker sent its done token (then return).
        worker: same wait (TF's join never returns; returning lets tasks exit)."""
        _log.info(f"[{self.job_name}:{self.task_index}] join: waiting for {self.rdv.num_workers} worker(s)")

        def on_dead(dead):
            _log.warning(f"[{self.job_name}:{self.task_index}] no heartbeat from worker(s) {dead}")
        try:
            ok = self.rdv.wait_all_workers_done(timeout=timeout, on_dead=on_dead)
        except Exception:      # store gone: the chief has already exited
            ok = True
        _log.info(f"[{self.job_name}:{self.task_index}] join finished ({'all done' if ok else 'timeout'})")
        self._leave()
        return ok

    def _leave(self):
        self.rdv.stop_heartbeat()
        try:
            self.rdv.store.set(f"left/{self.job_name}/{self.task_index}", b"1")
        except Exception:
            pass

    def signal_done(self, linger_s: float = 60.0):
        """Worker finished: done token for the ps.  The chief hosts the store,
        so it lingers until every other task has left (bounded by linger_s)."""
        if self._done or not self.rdv.is_worker:
            return
        self._done = True
        try:
            self.rdv.signal_done()
        except Exception:
            return
        if not self.is_chief:
            self._leave()
            return
        others = [f"left/{j}/{i}" for j in self.cluster.jobs for i in range(self.cluster.num_tasks(j))
                  if not (j == self.job_name and i == self.task_index)]
        t0 = time.time()
        while time.time() - t0 < linger_s:
            try:
                if not others or self.rdv.store.check(others):
                    break
            except Exception:
                break
            time.sleep(0.1)
        self.rdv.stop_heartbeat()

    def _atexit(self):
        self.signal_done()

    @staticmethod
    def create_local_server(config=None, start=True):
        from ..parallel.cluster import ClusterSpec as CS

        import socket

        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        return Server(CS({"worker": [f"127.0.0.1:{port}"]}), "worker", 0)


def current_server() -> Optional[Server]:
    return _SERVER


def _world_or_local():
    w = _world._WORLD
    return w if w is not None else _world.World(device=get_default_graph().device)


# ======================================================================= placement
def replica_device_setter(ps_tasks: int = 0, ps_device: str = "/job:ps", worker_device: str = "/job:worker",
                          merge_devices: bool = True, cluster=None, ps_ops=None, ps_strategy=None):
    """Returns the placement function of tf.train.replica_device_setter:
    variables round-robin over ps tasks, everything else on worker_device.
    The placement is recorded on each Variable (`.placement`) -- under sync DP
    dense variables are replicated on every worker's GPU and all-reduced, and
    `parallel.sharded_embedding` row-shards the huge ones across workers."""
    if cluster is not None:
        cs = cluster if isinstance(cluster, ClusterSpec) else ClusterSpec(cluster)
        ps_tasks = cs.num_tasks("ps")
    ps_ops = ps_ops or ["Variable", "VariableV2", "VarHandleOp", "AutoReloadVariable", "MutableHashTable"]
    state = {"next": 0}

    def place(op):
        if ps_tasks and getattr(op, "type", "") in ps_ops:
            if ps_strategy is not None:
                k = ps_strategy(op)
            else:
                k = state["next"] % ps_tasks
                state["next"] += 1
            return f"{ps_device}/task:{k}"
        return worker_device
    place.ps_tasks = ps_tasks
    return place


# ======================================================================= global step
def create_global_step(graph=None) -> Variable:
    g = get_default_graph()
    if g.get_collection(GLOBAL_STEP):
        raise ValueError("global_step already exists")
    v = get_variable("global_step", [], dtype=torch.int64, initializer=constant_initializer(0), trainable=False)
    g.add_to_collection(GLOBAL_STEP, v)
    return v


def get_global_step(graph=None) -> Optional[Variable]:
    g = get_default_graph()
    c = g.get_collection(GLOBAL_STEP)
    if c:
        return c[0]
    v = g._vars_by_name.get("global_step")
    return v


def get_or_create_global_step(graph=None) -> Variable:
    return get_global_step() or create_global_step()


def global_step(sess, global_step_tensor) -> int:
    return int(np.asarray(sess.run(global_step_tensor)))


# ======================================================================= gradient sync
def _is_pv(v) -> bool:
    return getattr(v, "is_partitioned", False)


class _GradSync:
    """Flat-bucket all-reduce (average) of a var_list's gradients across workers.

    The bucket is one flat fp32 buffer; gradients already written into its
    views (the lowered step's kernels write there directly) are not copied.
    A bf16/fp16 `comm_dtype` goes through the K16 pack + cast + 1/N kernel into
    a persistent 16-bit buffer and back (parallel/ddp.py's bucket kernels).
    With plain SGD on the node's IPC data plane the all-reduce and the update
    are ONE kernel (`sgd`, csrc/kernels/ipc_coll.hip reduce_sgd_k)."""

    def __init__(self, params: List[torch.Tensor], comm_dtype=None):
        self.params = params
        self.sizes = [p.numel() for p in params]
        self.n = sum(self.sizes)
        self.flat = torch.zeros(self.n, dtype=torch.float32, device=params[0].device)
        self.views = []
        off = 0
        for p, n in zip(params, self.sizes):
            self.views.append(self.flat[off:off + n].view_as(p))
            off += n
        self.comm_dtype = comm_dtype
        self.comm_buf = None

    def pack(self, grads: List[Optional[torch.Tensor]]):
        for v, g in zip(self.views, grads):
            if g is None:
                v.zero_()
            elif g is v or (g.data_ptr() == v.data_ptr() and g.shape == v.shape and g.stride() == v.stride()):
                continue                                  # written in place by the producer
            else:
                v.copy_(g)

    def __call__(self, grads: List[Optional[torch.Tensor]]) -> List[torch.Tensor]:
        with torch.no_grad():
            self.pack(grads)
            w = _world_or_local()
            if w.world_size > 1:
                flat = self.flat[:self.n]
                if self.comm_dtype in (torch.bfloat16, torch.float16) and flat.is_cuda:
                    from .. import _native
                    C = _native.load()
                    if self.comm_buf is None:
                        self.comm_buf = torch.empty(self.n, dtype=self.comm_dtype, device=flat.device)
                    C.bucket_pack(flat, self.comm_buf, 1.0 / w.world_size)     # K16: 1/N + cast in one pass
                    w.all_reduce(self.comm_buf, "sum")
                    C.bucket_unpack(self.comm_buf, flat, 1.0)
                elif flat.is_cuda:
                    w.all_reduce(flat, "avg")             # mean inside the collective: no extra pass
                else:
                    w.all_reduce(flat, "sum")
                    flat.mul_(1.0 / w.world_size)         # mean over workers == global-batch gradient
        return self.views

    def sgd(self, grads: List[Optional[torch.Tensor]], lr: float, global_step=None) -> Optional[bool]:
        """Synchronous SGD step as ONE kernel on the IPC data plane: every worker
        sums the W gradients in rank order (bit-identical replicas) and applies
        p -= lr / W * sum to its parameters; global_step += 1 inside it when the
        variable is a GPU scalar.  Returns None when not applicable (one worker,
        CPU, a 16-bit comm dtype, a plane other than IPC) -- a decision every
        rank makes alike; else whether global_step was advanced."""
        w = _world_or_local()
        if (w.world_size == 1 or not self.flat.is_cuda or self.comm_dtype not in (None, torch.float32)
                or len(self.params) > 8 or not all(p.dtype == torch.float32 and p.is_contiguous()
                                                   for p in self.params)):
            return None
        coll = w.gpu_coll(self.n * 4)               # collective on first use
        if coll is None or coll is not w.ipc or self.n * 4 > coll.capacity():
            return None
        with torch.no_grad():
            self.pack(grads)
            gv = getattr(global_step, "value", None) if global_step is not None else None
            gs = gv.data if (isinstance(gv, torch.Tensor) and gv.is_cuda and gv.numel() == 1 and gv.is_contiguous()
                             and gv.dtype in (torch.float32, torch.int64, torch.int32, torch.float64)) else None
            coll.reduce_sgd(self.flat, [p.data for p in self.params], lr_val=float(lr), gstep=gs)
        return gs is not None


# ======================================================================= optimizers
class Optimizer:
    """Base: compute_gradients / apply_gradients / minimize over compat Variables.

    `minimize` returns an Operation; running it performs one synchronous step:
    forward (memoised with other fetches of the same run), backward,
    all-reduce of the gradients across workers, fused optimizer update,
    global_step += 1."""

    _kind = "sgd"
    _slot_names: Sequence[str] = ()

    def __init__(self, learning_rate, use_locking=False, name=None, update_mode=None, **kw):
        self.learning_rate = learning_rate
        self.name = name or type(self).__name__.replace("Optimizer", "")
        self._kw = kw
        self.use_locking = bool(use_locking)
        # 'sync' (default: all-reduce data parallelism, the north star) or 'async'
        # (the reference's Hogwild ps updates, parallel/async_ps.py); None: $DTF_UPDATE_MODE
        self.update_mode = update_mode
        self.sync_replicas = True
        self.comm_dtype = None
        self._steps = 0

    def _make_fused(self, params):
        lr = float(self._lr_value())
        return _optim.FusedSGD(params, lr)

    def _lr_value(self):
        lr = self.learning_rate
        if isinstance(lr, Tensor):
            v = RunContext({}, get_default_graph().device).eval(lr)
            return float(v.detach().cpu()) if isinstance(v, torch.Tensor) else float(v)
        return float(lr)

    def compute_gradients(self, loss, var_list=None, **kw):
        """Dense variables get dense gradients; a PartitionedVariable gets the
        list of (lookup state, gradient rows) of the run -- TF's IndexedSlices."""
        var_list = list(var_list if var_list is not None else trainable_variables())
        key = id(loss)

        def grads_of(ctx):
            st = ctx.state.setdefault("grads", {})
            if key not in st:
                l = ctx.eval(loss)
                dense = [v for v in var_list if not _is_pv(v)]
                looks = [(pv, stt) for pv, stt in ctx.state.get("pv_lookups", []) if any(pv is v for v in var_list)]
                rows = [stt[0] for _, stt in looks]
                gs = torch.autograd.grad(l, [v.value for v in dense] + rows, allow_unused=True)
                dg = dict(zip(map(id, dense), gs[:len(dense)]))
                sparse = {}
                for (pv, stt), g in zip(looks, gs[len(dense):]):
                    sparse.setdefault(id(pv), []).append((stt[1], g))
                st[key] = [sparse.get(id(v), []) if _is_pv(v) else dg[id(v)] for v in var_list]
            return st[key]
        pairs = []
        for i, v in enumerate(var_list):
            t = Tensor(None, [], "gradients")
            t._eval = (lambda ctx, i=i: grads_of(ctx)[i])
            pairs.append((t, v))
        return pairs

    def apply_gradients(self, grads_and_vars, global_step=None, name=None) -> Operation:
        pairs = list(grads_and_vars)
        dense_pairs = [(g, v) for g, v in pairs if not _is_pv(v)]
        sparse_pairs = [(g, v) for g, v in pairs if _is_pv(v)]
        if sparse_pairs and self._kind not in ("sgd", "momentum", "adagrad", "rmsprop", "adam"):
            raise NotImplementedError(f"{type(self).__name__}: no sparse (partitioned-variable) update rule")
        for _, pv in sparse_pairs:      # owner-side sparse rule + sharded slots (TF names var/<slot>)
            pv.table.set_optimizer(self._kind, **self._sparse_hp())
            self._register_pv_slots(pv)
        self._register_nonslot([v for _, v in dense_pairs], [pv for _, pv in sparse_pairs])
        vars_ = [v for _, v in dense_pairs]
        gtens = [g for g, _ in dense_pairs]
        opt = self
        params = [v.value for v in vars_]
        # slots exist as soon as the train op does (TF creates them in
        # minimize), so a Saver built afterwards checkpoints/restores them
        fused = opt._make_fused(params) if params else None
        if fused is not None:
            opt._register_slots(vars_, fused)
        sync = _GradSync(params, opt.comm_dtype) if params else None
        if _async_ps.update_mode(opt.update_mode) == "async":
            return self._apply_async(vars_, gtens, params, sparse_pairs, global_step, name)

        def run(ctx):
            w = _world_or_local()
            ws = w.world_size
            opt._steps += 1
            _debug.fault_point(opt._steps, w.rank)
            gs_done = False
            fused_sgd = fused is not None and type(opt) is GradientDescentOptimizer and opt.sync_replicas
            if fused is not None:
                with _prof.range("compute_gradients"):
                    gs = [ctx.eval(g) if g is not None else None for g in gtens]
                done = sync.sgd(gs, opt._lr_value(), global_step) if fused_sgd else None
                if done is not None:
                    gs_done = done                  # all-reduce + update in one IPC kernel
                elif opt.sync_replicas:
                    with _prof.range("allreduce"):
                        gs = sync(gs)
                else:
                    gs = [g if g is not None else torch.zeros_like(p) for g, p in zip(gs, params)]
                if done is None:
                    if isinstance(opt.learning_rate, Tensor):
                        fused.set_lr(opt._lr_value())
                    fused.step(grads=[g.contiguous() for g in gs])
            lr = opt._lr_value()
            for g, pv in sparse_pairs:      # owner-side sparse update, sync average as grad_scale
                looks = ctx.eval(g)
                # several lookups of one variable: TF sums their IndexedSlices and
                # applies the rule once (SGD is linear, the others are not)
                multi = len(looks) > 1
                if multi:
                    pv.table.begin_update()
                for lctx, rows_grad in looks:
                    pv.table.apply_sgd(lctx, rows_grad if rows_grad is not None else
                                       torch.zeros((lctx.uniq.numel(), pv.dim), device=pv.table.device), lr,
                                       grad_scale=1.0 / ws)
                if multi:
                    pv.table.finish_update(lr)
            if global_step is not None and not gs_done:
                with torch.no_grad():
                    global_step.value.data += 1
            n = _debug.check_every()
            if n and opt._steps % n == 0:
                _debug.assert_replicas_consistent(w, params + [p.value for _, p in sparse_pairs], opt.name)
            return None
        op = Operation(None, [], name or self.name)
        op._eval = run
        # what compat/lowering.py needs to replace forward+backward (+ SGD) of
        # this op by fused kernels
        op._lowering = {"opt": opt, "vars": vars_, "fused": fused, "sync": sync, "global_step": global_step,
                        "sparse": sparse_pairs}
        return op

    def _apply_async(self, vars_, gtens, params, sparse_pairs, global_step, name) -> Operation:
        """The reference's asynchronous update (example.py:106-118 without
        SyncReplicasOptimizer; lr2.py:359-396's ps-held W trained by ScatterSub):
        pull the dense ps variables, gradient of this worker's batch, `var -= lr
        * grad` on the ps variables with no waiting; partitioned variables read
        their rows from -- and scatter their sparse updates into -- the owners'
        shared shards (HogwildTable); global_step = every worker's updates so
        far (parallel/async_ps.py)."""
        if self._kind != "sgd":
            raise NotImplementedError("asynchronous (Hogwild) updates: GradientDescentOptimizer only "
                                      "(update_mode='sync' handles the other optimizers)")
        opt = self
        state = {}

        def ensure():
            # collective: every worker's first train run, before its first forward
            # (the partitioned variables' lookups must already read the shared shards)
            if "store" in state:
                return
            w = _world_or_local()
            dense = params if params else [torch.zeros(1, device=sparse_pairs[0][1].table.device)]
            state["store"] = _async_ps.HogwildStore(dense, w, use_locking=opt.use_locking)
            for _, pv in sparse_pairs:
                if pv.table.hogwild is None:
                    pv.table.hogwild = _async_ps.HogwildTable(pv.table, w, use_locking=opt.use_locking)

        def pre_run():
            ensure()
            state["store"].pull()

        def run(ctx):
            w = _world_or_local()
            opt._steps += 1
            _debug.fault_point(opt._steps, w.rank)
            ensure()
            store = state["store"]
            lr = opt._lr_value()
            with _prof.range("compute_gradients"):
                gs = [ctx.eval(g) if g is not None else None for g in gtens]
                sgs = [(pv, ctx.eval(g)) for g, pv in sparse_pairs]
            with _prof.range("hogwild_update"):
                for pv, looks in sgs:       # owner-side scatter SGD into the shared shards, no waiting
                    for lctx, rows_grad in looks:
                        if rows_grad is not None:
                            pv.table.apply_sgd(lctx, rows_grad, lr)
                gstep = store.sgd_step(gs if params else [None], lr)
            if global_step is not None:
                with torch.no_grad():
                    global_step.value.data.fill_(float(gstep))
            return None
        op = Operation(None, [], name or self.name)
        op._eval = run
        op._async_state = state
        # Session.run calls this before evaluating anything: the forward of this
        # run reads the ps variables as they are now (other workers' updates included)
        op._pre_run = pre_run
        return op

    def minimize(self, loss, global_step=None, var_list=None, name=None, **kw) -> Operation:
        op = self.apply_gradients(self.compute_gradients(loss, var_list), global_step=global_step, name=name)
        op.loss = loss
        return op

    def _sparse_hp(self) -> dict:
        """Hyper-parameters of this optimizer's sparse (sharded-table) rule."""
        return {}

    def _register_pv_slots(self, pv):
        """A partitioned variable's slots: partitioned variables themselves
        (saved / restored in the TF slice layout like the table)."""
        from .partitioned import PartitionedSlot

        g = get_default_graph()
        names = {v.name for v in g.get_collection(GLOBAL_VARIABLES)}
        for sname in pv.table.slots:
            sv = PartitionedSlot(pv, sname)
            if sv.name not in names:
                g.add_to_collection(GLOBAL_VARIABLES, sv)

    # slot variables with TF names (w/Adam, w/Adam_1, beta1_power, ...) for checkpoints
    def _register_slots(self, vars_, fused):
        g = get_default_graph()
        for i, v in enumerate(vars_):
            base = v.name[:-2]
            for sname, tens in zip(self._slot_names, (fused.m[i], fused.v[i])):
                if tens is None:
                    continue
                sv = _SlotVariable(f"{base}/{sname}", tens, self._slot_init(sname))
                g.add_to_collection(GLOBAL_VARIABLES, sv)

    def get_slot_names(self):
        return list(self._slot_names)

    def _register_nonslot(self, dense_vars, pvs):
        """TF's non-slot optimizer variables (Adam: beta1_power / beta2_power)."""

    def _slot_init(self, sname: str) -> float:
        """Initial value TF gives the slot (zeros unless the optimizer says otherwise)."""
        return 0.0


class _SlotVariable:
    op_type, attrs = "VariableV2", {}       # a VariableV2 node in the exported GraphDef

    def __init__(self, name, tensor, init: float = 0.0):
        self.name = name + ":0"
        self.value = tensor
        self.init = float(init)
        self.initialized = True
        self.trainable = False

    def _initialize(self):
        with torch.no_grad():
            self.value.fill_(self.init)


class GradientDescentOptimizer(Optimizer):
    def _make_fused(self, params):
        return _optim.FusedSGD(params, self._lr_value())


class MomentumOptimizer(Optimizer):
    _kind = "momentum"
    _slot_names = ("Momentum",)

    def __init__(self, learning_rate, momentum, use_locking=False, name="Momentum", use_nesterov=False):
        super().__init__(learning_rate, use_locking, name)
        self.momentum, self.nesterov = momentum, use_nesterov

    def _make_fused(self, params):
        return _optim.FusedMomentum(params, self._lr_value(), self.momentum, self.nesterov)

    def _sparse_hp(self):
        return {"momentum": float(self.momentum), "use_nesterov": bool(self.nesterov)}


class AdamOptimizer(Optimizer):
    _kind = "adam"
    _slot_names = ("Adam", "Adam_1")

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, use_locking=False,
                 name="Adam"):
        super().__init__(learning_rate, use_locking, name)
        self.beta1, self.beta2, self.epsilon = beta1, beta2, epsilon

    def _make_fused(self, params):
        return _optim.FusedAdam(params, self._lr_value(), self.beta1, self.beta2, self.epsilon)

    def _sparse_hp(self):
        return {"beta1": float(self.beta1), "beta2": float(self.beta2), "epsilon": float(self.epsilon)}

    def _register_nonslot(self, dense_vars, pvs):
        # TF's non-slot accumulators beta1_power / beta2_power (= beta^(t+1)),
        # tied to the step count of the dense fused Adam and of every
        # partitioned variable's sparse Adam (a restore sets them all)
        steps = []
        for pv in pvs:
            if pv.table._adam is not None:
                steps.append(pv.table._adam.step_t)
        self._pending_powers = steps
        if not dense_vars and steps:
            self._add_powers(None)

    def _register_slots(self, vars_, fused):
        super()._register_slots(vars_, fused)
        self._add_powers(fused)

    def _add_powers(self, fused):
        g = get_default_graph()
        steps = ([fused.step_t] if fused is not None else []) + list(getattr(self, "_pending_powers", []))
        have = {v.name: v for v in g.get_collection(GLOBAL_VARIABLES)}
        for name, beta in (("beta1_power", self.beta1), ("beta2_power", self.beta2)):
            v = have.get(name + ":0")
            if isinstance(v, _PowerVariable):
                v.steps += [t for t in steps if all(t is not u for u in v.steps)]
            else:
                g.add_to_collection(GLOBAL_VARIABLES, _PowerVariable(name, beta, steps))
        p1, p2 = have.get("beta1_power:0"), have.get("beta2_power:0")
        if p1 is None or p2 is None:
            cur = {v.name: v for v in g.get_collection(GLOBAL_VARIABLES)}
            p1, p2 = cur.get("beta1_power:0"), cur.get("beta2_power:0")
        if isinstance(p1, _PowerVariable) and isinstance(p2, _PowerVariable):
            p1.sibling, p2.sibling = p2, p1


class _PowerVariable:
    """beta^(t+1) as a saveable variable, tied to the optimizers' step counts
    (`steps`: device int64 [1] tensors advanced together)."""

    op_type, attrs, shape, dtype = "VariableV2", {}, (), torch.float32

    def __init__(self, name, beta, steps):
        self.name = name + ":0"
        self.beta = beta
        self.steps = list(steps)
        self.initialized = True
        self._buf = torch.zeros((), dtype=torch.float32)
        self.sibling = None      # the other power of the same optimizer (beta1 <-> beta2)
        self._restored = None    # value read by the last restore

    @property
    def value(self):
        t = int(self.steps[0].item()) if self.steps else 0
        self._buf.fill_(self.beta ** (t + 1))  # TF stores beta^(t+1) after t updates
        return self._buf

    def restore_from(self, t: torch.Tensor):
        """Saver.restore: beta^(t+1) -> the step count of every tied optimizer.

        Uses both powers whichever order they are restored in: a power that
        underflowed (subnormal / 0 in float32) only bounds the count, the other
        one pins it (`optim.adam_steps_from_powers`)."""
        from ..optim import adam_steps_from_powers

        self._restored = float(t.reshape(-1)[0])
        sib = self.sibling
        other = (sib._restored, sib.beta) if sib is not None and sib._restored is not None else (None, None)
        steps = adam_steps_from_powers(self._restored, self.beta, *other)
        for s in self.steps:
            s.fill_(steps)

    def _initialize(self):
        for s in self.steps:
            s.zero_()


class AdagradOptimizer(Optimizer):
    _kind = "adagrad"
    _slot_names = ("Adagrad",)

    def __init__(self, learning_rate, initial_accumulator_value=0.1, use_locking=False, name="Adagrad"):
        super().__init__(learning_rate, use_locking, name)
        self.init_acc = initial_accumulator_value

    def _make_fused(self, params):
        return _optim.FusedAdagrad(params, self._lr_value(), self.init_acc)

    def _sparse_hp(self):
        return {"initial_accumulator_value": float(self.init_acc)}

    def _slot_init(self, sname: str) -> float:
        return float(self.init_acc)


class RMSPropOptimizer(Optimizer):
    _kind = "rmsprop"
    _slot_names = ("RMSProp", "Momentum")

    def __init__(self, learning_rate, decay=0.9, momentum=0.0, epsilon=1e-10, use_locking=False,
                 centered=False, name="RMSProp"):
        super().__init__(learning_rate, use_locking, name)
        if centered:
            raise NotImplementedError("RMSPropOptimizer(centered=True) is not supported")
        self.decay, self.mom, self.eps = decay, momentum, epsilon

    def _make_fused(self, params):
        return _optim.FusedRMSProp(params, self._lr_value(), self.decay, self.mom, self.eps)

    def _sparse_hp(self):
        return {"decay": float(self.decay), "momentum": float(self.mom), "epsilon": float(self.eps)}

    def _slot_init(self, sname: str) -> float:
        return 1.0 if sname == "RMSProp" else 0.0      # TF initialises the mean square to ones


class SyncReplicasOptimizer(Optimizer):
    """tf.train.SyncReplicasOptimizer (the commented path of example.py:109-123).

    Aggregation is an all-reduce over the workers; `replicas_to_aggregate` must
    equal the number of workers (backup workers / stale-gradient dropping are
    not modelled: every step is fully synchronous)."""

    def __init__(self, opt: Optimizer, replicas_to_aggregate: int, total_num_replicas: int = None,
                 replica_id: int = None, variable_averages=None, variables_to_average=None,
                 use_locking=False, name="sync_replicas"):
        super().__init__(opt.learning_rate, use_locking, name)
        self.opt = opt
        self.replicas_to_aggregate = replicas_to_aggregate
        self.total_num_replicas = total_num_replicas or replicas_to_aggregate
        w = _world._WORLD
        if w is not None and w.world_size > 1 and replicas_to_aggregate != w.world_size:
            _log.warning(f"SyncReplicasOptimizer: replicas_to_aggregate={replicas_to_aggregate} but "
                         f"{w.world_size} workers; all workers are aggregated every step")

    def compute_gradients(self, *a, **kw):
        return self.opt.compute_gradients(*a, **kw)

    def apply_gradients(self, grads_and_vars, global_step=None, name=None):
        self.opt.sync_replicas = True
        self.opt.update_mode = "sync"     # aggregation is the point of this wrapper
        return self.opt.apply_gradients(grads_and_vars, global_step, name)

    def get_init_tokens_op(self, num_tokens=-1):
        return Operation(lambda: None, [], "sync_token_init")

    def get_chief_queue_runner(self):
        return QueueRunner(None, [])

    def make_session_run_hook(self, is_chief, num_tokens=-1):
        return SessionRunHook()


# ======================================================================= init / sync helpers
def _broadcast_variables(vars_):
    w = _world_or_local()
    if w.world_size <= 1:
        return
    with torch.no_grad():
        for v in vars_:
            val = v.value
            if isinstance(val, torch.Tensor):
                w.broadcast(val.data, 0)


def _init_or_restore(sess, is_chief, init_op, local_init_op, init_fn, checkpoint_dir, saver, init_feed_dict):
    restored = None
    if checkpoint_dir:
        ck = latest_checkpoint(checkpoint_dir)
        if ck:
            (saver or Saver()).restore(sess, ck)
            restored = ck
    if restored is None:
        if is_chief:
            if init_op is not None:
                sess.run(init_op, feed_dict=init_feed_dict)
            else:
                for v in global_variables():
                    v._initialize()
            if init_fn is not None:
                init_fn(sess)
    # non-chief workers receive the chief's values (no re-initialisation race);
    # sharded (partitioned) variables are owned per rank: each initialises its shard
    if restored is None and not is_chief:
        for v in global_variables():
            if _is_pv(v):
                v._initialize()
    _broadcast_variables([v for v in global_variables() if isinstance(v, Variable) and not _is_pv(v)])
    for v in global_variables():
        if isinstance(v, Variable):
            v.initialized = True
    if local_init_op is not None:
        sess.run(local_init_op)
    else:
        for v in local_variables():
            v._initialize()
    return restored


# ======================================================================= Supervisor
class Supervisor:
    USE_DEFAULT = object()

    def __init__(self, graph=None, ready_op=USE_DEFAULT, is_chief=True, init_op=USE_DEFAULT,
                 init_feed_dict=None, local_init_op=USE_DEFAULT, logdir=None, summary_op=USE_DEFAULT,
                 saver=USE_DEFAULT, global_step=USE_DEFAULT, save_summaries_secs=120, save_model_secs=600,
                 recovery_wait_secs=30, stop_grace_secs=120, checkpoint_basename="model.ckpt",
                 session_manager=None, summary_writer=USE_DEFAULT, init_fn=None, **kw):
        self.is_chief = is_chief
        self.init_op = None if init_op is self.USE_DEFAULT else init_op
        if isinstance(self.init_op, (list, tuple)):
            from .graph import group

            self.init_op = group(*self.init_op)
        self.local_init_op = None if local_init_op is self.USE_DEFAULT else local_init_op
        self.init_feed_dict = init_feed_dict
        self.init_fn = init_fn
        self.logdir = logdir
        self.global_step = get_global_step() if global_step is self.USE_DEFAULT else global_step
        self.saver = (Saver() if logdir else None) if saver is self.USE_DEFAULT else saver
        self.summary_op = None if summary_op is self.USE_DEFAULT else summary_op
        self.save_model_secs = save_model_secs
        self.save_model_steps = int(kw.pop("save_model_steps", 0) or 0)
        self._last_saved = None
        self.save_summaries_secs = save_summaries_secs
        self.checkpoint_basename = checkpoint_basename
        self.coord = Coordinator()
        self.summary_writer = None
        if logdir and is_chief and summary_writer is self.USE_DEFAULT:
            self.summary_writer = FileWriter(logdir, get_default_graph())
        elif summary_writer not in (self.USE_DEFAULT, None):
            self.summary_writer = summary_writer
        self._threads: List[threading.Thread] = []
        self._sess = None
        self.save_path = os.path.join(logdir, checkpoint_basename) if logdir else None

    def prepare_or_wait_for_session(self, master="", config=None, wait_for_checkpoint=False,
                                    max_wait_secs=7200, start_standard_services=True) -> Session:
        sess = Session(master, config=config)
        _init_or_restore(sess, self.is_chief, self.init_op, self.local_init_op, self.init_fn,
                         self.logdir, self.saver, self.init_feed_dict)
        self._sess = sess
        if start_standard_services and self.logdir:
            self._start_services(sess)
        return sess

    def _collective_save(self) -> bool:
        """Sharded (partitioned) variables make a save collective: every rank
        writes its shard.  Otherwise only the chief writes."""
        w = _world._WORLD
        return w is not None and w.world_size > 1 and any(_is_pv(v) for v in global_variables())

    def _save(self, sess):
        self.saver.save(sess, self.save_path, global_step=self._gstep(sess))

    def _start_services(self, sess):
        """Checkpoints are taken at step boundaries by a post-run callback in the
        training thread (a timer only raises the flag): a checkpoint never mixes
        parameters of two steps.  `save_model_steps` (extension) gives a
        deterministic cadence every rank agrees on -- required for collective
        saves of sharded tables."""
        if self.saver is not None and (self.save_model_secs or self.save_model_steps):
            collective = self._collective_save()
            if self.save_model_steps:
                def on_step(s):
                    g = self._gstep(s)
                    if g and g % self.save_model_steps == 0 and g != self._last_saved:
                        self._last_saved = g
                        self._save(s)
                sess._post_run.append(on_step)
            elif self.is_chief and not collective:
                due = threading.Event()

                def timer():
                    while not self.coord.wait_for_stop(self.save_model_secs):
                        due.set()
                t = threading.Thread(target=timer, daemon=True, name="sv-checkpoint-timer")
                t.start()
                self._threads.append(t)

                def on_run(s):
                    if due.is_set():
                        due.clear()
                        self._save(s)
                sess._post_run.append(on_run)
        if self.is_chief and self.summary_op is not None and self.summary_writer is not None and \
                self.save_summaries_secs:
            def sum_loop():
                while not self.coord.wait_for_stop(self.save_summaries_secs):
                    try:
                        self.summary_writer.add_summary(sess.run(self.summary_op), self._gstep(sess))
                    except Exception:
                        pass
            t = threading.Thread(target=sum_loop, daemon=True, name="sv-summary")
            t.start()
            self._threads.append(t)

    def _gstep(self, sess):
        gs = self.global_step
        if gs is None:
            return None
        if isinstance(gs, Variable):          # readable after the session closed (sv.stop())
            return int(float(gs.value.detach().reshape(-1)[0]))
        return int(np.asarray(sess.run(gs)))

    @contextlib.contextmanager
    def managed_session(self, master="", config=None, start_standard_services=True, close_summary_writer=True):
        sess = self.prepare_or_wait_for_session(master, config, start_standard_services=start_standard_services)
        try:
            yield sess
        except Exception as e:
            self.coord.request_stop(e)
            raise
        finally:
            self.stop(close_summary_writer=close_summary_writer)

    def start_queue_runners(self, sess, queue_runners=None):
        threads = []
        for qr in (queue_runners or get_default_graph().get_collection("queue_runners")):
            threads += qr.create_threads(sess, coord=self.coord, daemon=True, start=True)
        return threads

    def summary_computed(self, sess, summary, global_step=None):
        if self.summary_writer is not None:
            self.summary_writer.add_summary(summary, global_step if global_step is not None else self._gstep(sess))

    def should_stop(self):
        return self.coord.should_stop()

    def request_stop(self, ex=None):
        self.coord.request_stop(ex)

    def stop(self, threads=None, close_summary_writer=True, ignore_live_threads=False):
        self.coord.request_stop()
        for t in self._threads:
            t.join(5)
        if self.saver is not None and self._sess is not None and self.logdir and \
                (self.is_chief or self._collective_save()):
            self._sess._post_run.clear()
            self._save(self._sess)
        if close_summary_writer and self.summary_writer is not None:
            self.summary_writer.close()
        srv = current_server()
        if srv is not None:
            srv.signal_done()

    def wait_for_stop(self):
        self.coord.wait_for_stop()

    @property
    def session_manager(self):
        return self


# ======================================================================= hooks
class SessionRunArgs:
    def __init__(self, fetches=None, feed_dict=None, options=None):
        self.fetches = fetches
        self.feed_dict = feed_dict
        self.options = options


class SessionRunValues:
    def __init__(self, results, options=None, run_metadata=None):
        self.results = results
        self.options = options
        self.run_metadata = run_metadata


class SessionRunContext:
    def __init__(self, original_args, session):
        self.original_args = original_args
        self.session = session
        self._stop = False

    def request_stop(self):
        self._stop = True

    @property
    def stop_requested(self):
        return self._stop


class SessionRunHook:
    def begin(self):
        pass

    def after_create_session(self, session, coord):
        pass

    def before_run(self, run_context):
        return None

    def after_run(self, run_context, run_values):
        pass

    def end(self, session):
        pass


class NanLossDuringTrainingError(RuntimeError):
    pass


class StopAtStepHook(SessionRunHook):
    def __init__(self, num_steps=None, last_step=None):
        if (num_steps is None) == (last_step is None):
            raise ValueError("exactly one of num_steps and last_step")
        self.num_steps, self.last_step = num_steps, last_step

    def after_create_session(self, session, coord):
        gs = get_global_step()
        cur = int(np.asarray(session.run(gs))) if gs is not None else 0
        if self.last_step is None:
            self.last_step = cur + self.num_steps

    def after_run(self, ctx, vals):
        gs = get_global_step()
        if gs is not None and int(np.asarray(ctx.session.run(gs))) >= self.last_step:
            ctx.request_stop()


class CheckpointSaverHook(SessionRunHook):
    def __init__(self, checkpoint_dir, save_secs=None, save_steps=None, saver=None,
                 checkpoint_basename="model.ckpt", scaffold=None, listeners=None):
        self.dir = checkpoint_dir
        self.save_secs, self.save_steps = save_secs, save_steps
        self.saver = saver
        self.path = os.path.join(checkpoint_dir, checkpoint_basename)
        self._last_t = time.time()
        self._last_step = None
        self.listeners = listeners or []

    def _gs(self, sess):
        gs = get_global_step()
        return int(np.asarray(sess.run(gs))) if gs is not None else 0

    def after_create_session(self, session, coord):
        self.saver = self.saver or Saver()
        self._last_step = self._gs(session)
        if not latest_checkpoint(self.dir):
            self.saver.save(session, self.path, global_step=self._last_step)

    def after_run(self, ctx, vals):
        step = self._gs(ctx.session)
        due = (self.save_steps and step - self._last_step >= self.save_steps) or \
              (self.save_secs and time.time() - self._last_t >= self.save_secs)
        if due:
            self.saver.save(ctx.session, self.path, global_step=step)
            self._last_step, self._last_t = step, time.time()
            for l in self.listeners:
                getattr(l, "after_save", lambda *a: None)(ctx.session, step)

    def end(self, session):
        step = self._gs(session)
        if step != self._last_step:
            self.saver.save(session, self.path, global_step=step)


class SummarySaverHook(SessionRunHook):
    def __init__(self, save_steps=None, save_secs=None, output_dir=None, summary_writer=None, scaffold=None,
                 summary_op=None):
        self.save_steps, self.save_secs = save_steps, save_secs
        self.writer = summary_writer or (FileWriter(output_dir) if output_dir else None)
        self.op = summary_op
        self._n = 0

    def before_run(self, ctx):
        op = self.op
        if op is None:
            from .summary import merge_all

            op = self.op = merge_all()
        due = op is not None and self.save_steps and self._n % self.save_steps == 0
        gs = get_global_step()
        return SessionRunArgs({"s": op if due else None, "g": gs})

    def after_run(self, ctx, vals):
        self._n += 1
        r = vals.results or {}
        if r.get("s") is not None and self.writer is not None:
            self.writer.add_summary(r["s"], int(np.asarray(r["g"])) if r.get("g") is not None else self._n)

    def end(self, session):
        if self.writer is not None:
            self.writer.flush()


class LoggingTensorHook(SessionRunHook):
    def __init__(self, tensors, every_n_iter=None, every_n_secs=None, at_end=False, formatter=None):
        self.tensors = tensors if isinstance(tensors, dict) else {getattr(t, "name", str(t)): t for t in tensors}
        self.n = every_n_iter or 1
        self._i = 0
        self.formatter = formatter

    def before_run(self, ctx):
        return SessionRunArgs(self.tensors) if self._i % self.n == 0 else None

    def after_run(self, ctx, vals):
        if vals.results:
            msg = self.formatter(vals.results) if self.formatter else ", ".join(
                f"{k} = {v}" for k, v in vals.results.items())
            _log.info(msg)
        self._i += 1


class NanTensorHook(SessionRunHook):
    def __init__(self, loss_tensor, fail_on_nan_loss=True):
        self.loss, self.fail = loss_tensor, fail_on_nan_loss

    def before_run(self, ctx):
        return SessionRunArgs(self.loss)

    def after_run(self, ctx, vals):
        if vals.results is not None and not np.all(np.isfinite(vals.results)):
            if self.fail:
                raise NanLossDuringTrainingError("NaN loss during training.")
            ctx.request_stop()


class StepCounterHook(SessionRunHook):
    def __init__(self, every_n_steps=100, every_n_secs=None, output_dir=None, summary_writer=None):
        self.n = every_n_steps
        self.writer = summary_writer or (FileWriter(output_dir) if output_dir else None)
        self._i, self._t = 0, time.time()

    def after_run(self, ctx, vals):
        self._i += 1
        if self._i % self.n == 0:
            dt = time.time() - self._t
            sps = self.n / max(dt, 1e-9)
            if self.writer is not None:
                self.writer.add_scalar("global_step/sec", sps, self._i)
            _log.info(f"global_step/sec: {sps:.2f}")
            self._t = time.time()


class FinalOpsHook(SessionRunHook):
    def __init__(self, final_ops, final_ops_feed_dict=None):
        self.final_ops, self.feed = final_ops, final_ops_feed_dict
        self.final_ops_values = None

    def end(self, session):
        self.final_ops_values = session.run(self.final_ops, feed_dict=self.feed)


# ======================================================================= MonitoredSession
class Scaffold:
    def __init__(self, init_op=None, init_feed_dict=None, init_fn=None, ready_op=None, local_init_op=None,
                 summary_op=None, saver=None):
        self.init_op, self.init_feed_dict, self.init_fn = init_op, init_feed_dict, init_fn
        self.local_init_op, self.summary_op, self.saver = local_init_op, summary_op, saver

    def finalize(self):
        return self


class MonitoredSession:
    def __init__(self, is_chief=True, checkpoint_dir=None, scaffold=None, hooks=None, master="", config=None):
        self.scaffold = scaffold or Scaffold()
        self.hooks = list(hooks or [])
        self._sess = Session(master, config=config)
        self.coord = Coordinator()
        for h in self.hooks:
            h.begin()
        _init_or_restore(self._sess, is_chief, self.scaffold.init_op, self.scaffold.local_init_op,
                         self.scaffold.init_fn, checkpoint_dir, self.scaffold.saver, self.scaffold.init_feed_dict)
        self._qr_threads = start_queue_runners(self._sess, self.coord)
        for h in self.hooks:
            h.after_create_session(self._sess, self.coord)
        self._stop = False
        self._closed = False

    @property
    def graph(self):
        return get_default_graph()

    def run(self, fetches, feed_dict=None, options=None, run_metadata=None):
        ctx = SessionRunContext(SessionRunArgs(fetches, feed_dict, options), self._sess)
        extra = [h.before_run(ctx) for h in self.hooks]
        merged_feed = dict(feed_dict or {})
        for e in extra:
            if e is not None and e.feed_dict:
                merged_feed.update(e.feed_dict)
        all_fetches = {"__main": fetches, "__hooks": [e.fetches if e is not None else None for e in extra]}
        res = self._sess.run(all_fetches, feed_dict=merged_feed, options=options)
        for h, e, r in zip(self.hooks, extra, res["__hooks"]):
            h.after_run(ctx, SessionRunValues(r if e is not None else None))
        if ctx.stop_requested:
            self._stop = True
        return res["__main"]

    def run_step_fn(self, step_fn):
        return step_fn(self)

    def should_stop(self) -> bool:
        return self._stop or self.coord.should_stop()

    def request_stop(self):
        self._stop = True

    def close(self):
        if self._closed:
            return
        self._closed = True
        for h in self.hooks:
            h.end(self._sess)
        self.coord.request_stop()
        self._sess.close()
        srv = current_server()
        if srv is not None:
            srv.signal_done()

    def __enter__(self):
        return self

    def __exit__(self, et, ev, tb):
        if ev is not None and not isinstance(ev, Exception):
            pass
        self.close()
        return False


SingularMonitoredSession = MonitoredSession


def MonitoredTrainingSession(master="", is_chief=True, checkpoint_dir=None, scaffold=None, hooks=None,  # noqa: N802
                             chief_only_hooks=None, save_checkpoint_secs=600, save_summaries_steps=100,
                             save_summaries_secs=None, config=None, stop_grace_period_secs=120,
                             log_step_count_steps=100, max_wait_secs=7200, save_checkpoint_steps=None,
                             summary_dir=None):
    """tf.train.MonitoredTrainingSession: chief restores-or-initialises and
    broadcasts, runs checkpoint / summary / step-counter hooks."""
    all_hooks = list(hooks or [])
    if is_chief:
        all_hooks += list(chief_only_hooks or [])
        sdir = summary_dir or checkpoint_dir
        if checkpoint_dir and (save_checkpoint_secs or save_checkpoint_steps):
            all_hooks.append(CheckpointSaverHook(checkpoint_dir, save_secs=save_checkpoint_secs,
                                                 save_steps=save_checkpoint_steps,
                                                 saver=(scaffold.saver if scaffold else None)))
        if sdir and save_summaries_steps:
            all_hooks.append(SummarySaverHook(save_steps=save_summaries_steps, output_dir=sdir,
                                              summary_op=(scaffold.summary_op if scaffold else None)))
        if sdir and log_step_count_steps:
            all_hooks.append(StepCounterHook(log_step_count_steps, output_dir=sdir))
    return MonitoredSession(is_chief, checkpoint_dir, scaffold, all_hooks, master, config)


# ======================================================================= lr schedules
def exponential_decay(learning_rate, global_step, decay_steps, decay_rate, staircase=False, name=None):
    def f(gs):
        p = float(gs) / decay_steps
        if staircase:
            p = float(int(p))
        return torch.tensor(learning_rate * decay_rate ** p)
    return Tensor(f, [global_step], name or "ExponentialDecay")


def piecewise_constant(x, boundaries, values, name=None):
    def f(v):
        v = float(v)
        for b, val in zip(boundaries, values):
            if v <= b:
                return torch.tensor(float(val))
        return torch.tensor(float(values[-1]))
    return Tensor(f, [x], name or "PiecewiseConstant")
