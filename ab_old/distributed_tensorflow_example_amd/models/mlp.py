"""The reference's headline model: 784-100-10 MLP trained with SGD
(example.py:69-128; sigmoid hidden layer, softmax output, mean cross-entropy,
GradientDescentOptimizer(0.0005), batch 100 per worker).

Three implementations of the same step:

* `reference_step`   -- plain PyTorch fp32 (the numerics oracle for the HIP
                        kernels, and the CPU/gloo path of BASELINE config #1).
* `MLP` (nn.Module)  -- generic path built from the framework ops
                        (`ops.linear_act`, `ops.softmax_xent`), used by the
                        TF-compat session layer and autograd users.
* `FusedMLPTrainer`  -- the MI355X hot path: 2 kernels per step on 1 GPU, or
                        2 kernels + one RCCL all-reduce + the flat SGD kernel
                        in sync data parallel (csrc/kernels/mlp_step.hip),
                        replayed from hipGraphs by `MLPStepRunner` with the
                        input streamed from pinned host memory on a side stream.

Parameter layout (flat fp32, TF variable order and names):
  weights/Variable [784,100], weights/Variable_1 [100,10],
  biases/Variable [100], biases/Variable_1 [10].
"""
from __future__ import annotations

import math
import os
import time
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import _native

D_IN, HIDDEN, N_CLS = 784, 100, 10
OFF_W1, OFF_W2, OFF_B1, OFF_B2 = 0, 78400, 79400, 79500
NPARAM = 79510
PARAM_SPECS: "OrderedDict[str, Tuple[int, Tuple[int, ...]]]" = OrderedDict([
    ("weights/Variable", (OFF_W1, (D_IN, HIDDEN))),
    ("weights/Variable_1", (OFF_W2, (HIDDEN, N_CLS))),
    ("biases/Variable", (OFF_B1, (HIDDEN,))),
    ("biases/Variable_1", (OFF_B2, (N_CLS,))),
])
ACTS = {"sigmoid": 0, "relu": 1}


def init_params(seed: int = 1) -> torch.Tensor:
    """W ~ N(0,1) (tf.random_normal, example.py:84-85), b = 0 (example.py:89-90)."""
    g = torch.Generator().manual_seed(seed)
    p = torch.zeros(NPARAM, dtype=torch.float32)
    p[OFF_W1:OFF_W2] = torch.randn(D_IN * HIDDEN, generator=g)
    p[OFF_W2:OFF_B1] = torch.randn(HIDDEN * N_CLS, generator=g)
    return p


def unflatten(flat: torch.Tensor) -> Dict[str, torch.Tensor]:
    out = {}
    for name, (off, shape) in PARAM_SPECS.items():
        n = int(np.prod(shape))
        out[name] = flat[off:off + n].view(*shape)
    return out


def _act(z, act):
    return torch.sigmoid(z) if act == "sigmoid" else torch.relu(z)


def reference_forward(flat: torch.Tensor, x: torch.Tensor, act: str = "sigmoid"):
    p = unflatten(flat)
    z2 = x @ p["weights/Variable"] + p["biases/Variable"]
    a2 = _act(z2, act)
    z3 = a2 @ p["weights/Variable_1"] + p["biases/Variable_1"]
    return z3


def reference_loss_and_grad(flat: torch.Tensor, x: torch.Tensor, labels: torch.Tensor,
                            act: str = "sigmoid", naive: bool = False):
    """fp32 loss, accuracy and flat gradient (autograd) of one batch."""
    w = flat.detach().clone().requires_grad_(True)
    z3 = reference_forward(w, x.float(), act)
    y = torch.nn.functional.one_hot(labels.long(), N_CLS).float()
    if naive:  # -sum(y * log(softmax)) exactly as example.py:103 (can be inf/NaN)
        loss = torch.mean(-torch.sum(y * torch.log(torch.softmax(z3, 1)), 1))
    else:
        loss = torch.nn.functional.cross_entropy(z3, labels.long())
    loss.backward()
    acc = (z3.argmax(1) == labels.long()).float().mean()
    return loss.detach(), acc.detach(), w.grad.detach()


def reference_step(flat: torch.Tensor, x: torch.Tensor, labels: torch.Tensor, lr: float,
                   act: str = "sigmoid"):
    loss, acc, g = reference_loss_and_grad(flat, x, labels, act)
    flat.sub_(lr * g)
    return loss, acc


class MLP(torch.nn.Module):
    """Generic-path MLP on the framework's fused ops (autograd-enabled)."""

    def __init__(self, act: str = "sigmoid", seed: int = 1, device=None):
        super().__init__()
        flat = init_params(seed)
        p = unflatten(flat)
        self.W1 = torch.nn.Parameter(p["weights/Variable"].clone())
        self.W2 = torch.nn.Parameter(p["weights/Variable_1"].clone())
        self.b1 = torch.nn.Parameter(p["biases/Variable"].clone())
        self.b2 = torch.nn.Parameter(p["biases/Variable_1"].clone())
        self.act = act
        if device is not None:
            self.to(device)

    def tf_variables(self) -> "OrderedDict[str, torch.nn.Parameter]":
        return OrderedDict([("weights/Variable", self.W1), ("weights/Variable_1", self.W2),
                            ("biases/Variable", self.b1), ("biases/Variable_1", self.b2)])

    def forward(self, x):
        from ..ops import linear_act

        a2 = linear_act(x, self.W1, self.b1, self.act)
        return linear_act(a2, self.W2, self.b2, "none")


class FusedMLPTrainer:
    """One rank's fused MLP training step (see module doc)."""

    def __init__(self, batch_size: int = 100, lr: float = 0.0005, act: str = "sigmoid",
                 world=None, grad_dtype: torch.dtype = torch.bfloat16, naive_loss: bool = False,
                 metrics_ring: int = 8192, seed: int = 1, device=None, allreduce: str = "auto",
                 ipc_timeout_s: float = 5.0):
        self.C = _native.load()
        self.world = world
        self.world_size = 1 if world is None else world.world_size
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        dev = self.device
        B = int(batch_size)
        self.B = B
        self.nb = (B + 15) // 16
        self.BP = ((B + 31) // 32) * 32
        self.act = ACTS[act]
        self.act_name = act
        self.naive = bool(naive_loss)
        bf = torch.bfloat16
        self.params = torch.zeros(NPARAM, dtype=torch.float32, device=dev)
        self.W1T = torch.zeros(112 * 800, dtype=bf, device=dev)
        self.W2T = torch.zeros(16 * 128, dtype=bf, device=dev)
        self.W2N = torch.zeros(112 * 32, dtype=bf, device=dev)
        self.z2p = torch.zeros(self.C.mlp_ksplit() * self.nb * 16 * 112, dtype=torch.float32,
                               device=dev)
        self.dz2T = torch.zeros(112 * self.BP, dtype=bf, device=dev)
        self.partials = torch.zeros(self.nb * 1112, dtype=torch.float32, device=dev)
        self.grad_dtype = grad_dtype
        self.grads = (torch.zeros(NPARAM, dtype=grad_dtype, device=dev)
                      if self.world_size > 1 else None)
        self.lr = torch.tensor([lr], dtype=torch.float32, device=dev)
        self.ring = int(metrics_ring)
        self.metrics = torch.zeros(self.ring * 2, dtype=torch.float32, device=dev)
        self.gstep = torch.zeros(1, dtype=torch.int64, device=dev)
        self.counters = torch.zeros(max(64, self.nb), dtype=torch.int32, device=dev)
        # A1+A2 merged by last-arriver handoff: correct, but measured 13.56 vs 13.16 us/step
        # for the split pair on MI355X (the split boundary is cheaper than the handoff), so opt-in
        self.merged_head = os.environ.get("DTF_MLP_MERGED_HEAD", "0") == "1"
        self.allreduce = "none"
        self.ipc = None
        self.ipc_parity = 0
        self.ipc_mode = None
        self.ipc_timeout_s = float(ipc_timeout_s)
        if self.world_size > 1 and allreduce == "external":
            # the caller owns the gradient exchange (PersistentMLPRunner: in-kernel
            # over IPC): no exchange buffers, no RCCL communicator
            self.allreduce = "external"
        elif self.world_size > 1:
            self.allreduce = "rccl"
            if allreduce in ("ipc", "ipc-fused", "ipc-apply", "auto"):
                try:
                    self._setup_ipc()
                    self.ipc_mode = "apply" if allreduce == "ipc-apply" else "fused"
                    self.allreduce = "ipc-" + self.ipc_mode
                except Exception as e:  # noqa: BLE001
                    if allreduce.startswith("ipc"):
                        raise
                    import warnings

                    warnings.warn(f"IPC all-reduce unavailable ({e}); using RCCL")
            if self.allreduce == "rccl":
                # created here, collectively, only when this trainer's exchange is RCCL
                # (RuntimeError if it cannot come up: the caller falls back)
                world.ensure_comm()
        # RCCL and the IPC kernels capture into hipGraphs; a gloo all-reduce (ranks
        # sharing one GPU in tests) does not
        self.graph_safe = (self.world_size == 1 or self.allreduce.startswith("ipc")
                           or (world is not None and world.comm is not None))
        self.shadows_stale = False   # set by PersistentMLPRunner (it updates only the fp32 master)
        self.set_params(init_params(seed))

    # ---------------------------------------------------------------- IPC one-shot all-reduce
    def _setup_ipc(self):
        """Map every rank's gradient buffer (xGMI peers of one node); handles go
        through the gloo control plane.  Layout: [flags][grad slot 0][grad slot 1]."""
        w = self.world
        if int(os.environ.get("LOCAL_WORLD_SIZE", w.world_size)) != w.world_size:
            raise RuntimeError("IPC all-reduce needs all ranks on one node")
        C = self.C
        self.ipc_flag_bytes = C.mlp_ipc_flag_bytes()
        self.ipc_slot = ((NPARAM * 2 + 255) // 256) * 256
        from ..parallel.world import open_peer_buffers
        buf = open_peer_buffers(C, self.ipc_flag_bytes + 2 * self.ipc_slot, w)
        self.ipc = buf
        self.ipc_grads = [buf.tensor(self.ipc_flag_bytes + p * self.ipc_slot, NPARAM, 1) for p in (0, 1)]
        self.ipc_err = torch.zeros(1, dtype=torch.int32, device=self.device)

    def ipc_error(self) -> int:
        return int(self.ipc_err.item()) if self.ipc is not None else 0

    # ---------------------------------------------------------------- state
    def set_params(self, flat_cpu: torch.Tensor, broadcast: bool = True):
        self.params.copy_(flat_cpu.to(self.device, torch.float32))
        if broadcast and self.world is not None and self.world_size > 1:
            self.world.broadcast(self.params, 0)  # chief init + broadcast
        self.refresh_shadows()

    def refresh_shadows(self):
        self.C.mlp_apply_flat(self.params, None, self.lr, 0.0, self.W1T, self.W2T, self.W2N)
        self.shadows_stale = False

    def get_params(self) -> torch.Tensor:
        return self.params.detach().cpu()

    def set_lr(self, lr: float):
        self.lr.fill_(lr)

    @property
    def global_step(self) -> int:
        return int(self.gstep.item())

    def set_global_step(self, v: int):
        self.gstep.fill_(int(v))

    def read_metrics(self, first_step: int, last_step: int) -> np.ndarray:
        """(loss, accuracy) rows for global steps [first, last)."""
        m = self.metrics.view(self.ring, 2).cpu().numpy()
        idx = np.arange(first_step, last_step) % self.ring
        return m[idx]

    # ----------------------------------------------------------------- steps
    def enqueue_step(self, x: torch.Tensor, x_off: int, x_kind: int, labels: torch.Tensor,
                     labels_off: int, ipc_parity: Optional[int] = None):
        """Enqueue one full training step on the current stream.

        x: device buffer holding B rows of 784 features at byte offset x_off
        (kind 0 uint8 pixels, 1 fp32, 2 bf16); labels: uint8 class ids.
        """
        C, B = self.C, self.B
        if self.shadows_stale:
            self.refresh_shadows()
        if self.merged_head:   # A1+A2 in one launch (last-arriver handoff per row block)
            C.mlp_fwd_head(x, x_off, x_kind, B, self.W1T, self.z2p, labels, labels_off, self.W2T, self.W2N,
                           self.params, self.dz2T, self.partials, 1.0 / B, self.act, self.naive, self.counters,
                           self.gstep)
        else:
            C.mlp_l1_fwd(x, x_off, x_kind, B, self.W1T, self.z2p)
            C.mlp_head_bwd(self.z2p, labels, labels_off, B, self.W2T, self.W2N, self.params, self.dz2T,
                           self.partials, 1.0 / B, self.act, self.naive, self.gstep)
        if self.world_size == 1:
            C.mlp_wgrad(x, x_off, x_kind, self.dz2T, B, self.partials, self.params, self.W1T,
                        self.W2T, self.W2N, None, 0, self.lr, self.metrics, self.gstep)
        elif self.ipc is not None:
            par = self.ipc_parity if ipc_parity is None else int(ipc_parity) & 1
            if ipc_parity is None:
                self.ipc_parity ^= 1
            if self.ipc_mode == "fused":
                # every wgrad workgroup swaps its gradient block with the same workgroup
                # on all peers (IPC over xGMI) and applies SGD in place: 3 launches/step
                C.mlp_wgrad(x, x_off, x_kind, self.dz2T, B, self.partials, self.params, self.W1T,
                            self.W2T, self.W2N, None, 3, self.lr, self.metrics, self.gstep, None,
                            self.ipc.table_ptr(), self.world_size, self.world.rank, par, self.ipc_slot,
                            self.ipc_err, self.ipc_timeout_s)
            else:
                # one-shot: bf16 grads into this rank's exported slot, then every rank
                # sums all peers' slots over xGMI inside the SGD apply kernel
                C.mlp_wgrad(x, x_off, x_kind, self.dz2T, B, self.partials, self.params, self.W1T,
                            self.W2T, self.W2N, self.ipc_grads[par], 2, self.lr, self.metrics, self.gstep)
                C.mlp_ipc_reduce_apply(self.params, self.ipc.table_ptr(), self.world_size, self.world.rank, par,
                                       self.ipc_slot, self.gstep, self.lr, 1.0 / self.world_size, self.W1T,
                                       self.W2T, self.W2N, self.ipc_err, self.ipc_timeout_s)
        else:
            kind = 1 if self.grad_dtype == torch.float32 else 2
            C.mlp_wgrad(x, x_off, x_kind, self.dz2T, B, self.partials, self.params, self.W1T,
                        self.W2T, self.W2N, self.grads, kind, self.lr, self.metrics, self.gstep)
            self.world.all_reduce(self.grads, "sum")
            C.mlp_apply_flat(self.params, self.grads, self.lr, 1.0 / self.world_size, self.W1T,
                             self.W2T, self.W2N)

    def step_tensors(self, x: torch.Tensor, labels: torch.Tensor):
        """Eager step on device tensors (x: uint8/fp32/bf16 [B,784], labels [B])."""
        kind = {torch.uint8: 0, torch.float32: 1, torch.bfloat16: 2}[x.dtype]
        self.enqueue_step(x.contiguous(), 0, kind, labels.to(torch.uint8).contiguous(), 0)


class GemmMLPTrainer:
    """Large-batch step of the same model (csrc/kernels/mlp_gemm.hip), 4
    launches: `mlpg_l1` (one workgroup per 64 rows x 16 hidden units: the
    hidden layer on bf16 MFMA with W1 as an exact 3-way bf16 split) and
    `mlpg_head` (one workgroup per 16 rows, its waves splitting the hidden
    tiles: logits, softmax-xent, dz2 and the dW2/db2 partials on exact-f32 MFMA),
    `mlpg_wgrad` ([dW1; db1] over a 64-pixel-block x 256-row-chunk grid, dz2 as
    its exact split) and `mlpg_apply` (fixed-order slab reduction, SGD, W1
    fragment-image refresh, metrics).  The fused engines contract the batch serially inside
    one wave per weight tile: right at B=100, 4x too slow at B=4096.  All three
    launches are graph-capturable, so `MLPStepRunner` replays them exactly like
    the fused trainer's.  N > 1: the apply kernel first writes the reduced flat
    fp32 gradient, one RCCL all-reduce, then the apply.

    Same interface as `FusedMLPTrainer` (params / metrics ring / global step)."""

    def __init__(self, batch_size: int = 4096, lr: float = 0.0005, act: str = "sigmoid", world=None,
                 naive_loss: bool = False, metrics_ring: int = 8192, seed: int = 1, device=None,
                 **_ignored):
        self.C = _native.load()
        self.world = world
        self.world_size = 1 if world is None else world.world_size
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        dev = self.device
        B = self.B = int(batch_size)
        self.BP = (B + 63) // 64 * 64
        self.act = ACTS[act]
        self.act_name = act
        self.naive = bool(naive_loss)
        f32 = torch.float32
        # dW1: one workgroup per (64-pixel block, 128- or 256-row batch chunk); the
        # B-fragment image of dz2 is padded (with zeros) to whole chunks
        wc = self.C.mlpg_wchunk(B)
        self.nchunk = (B + wc - 1) // wc
        self.params = torch.zeros(NPARAM, dtype=f32, device=dev)
        self.W1S = torch.zeros(3 * 112 * 800, dtype=torch.bfloat16, device=dev)
        self.dz2S = torch.zeros(3 * 112 * self.nchunk * wc, dtype=torch.bfloat16, device=dev)
        self.a2 = torch.zeros(self.BP * 112, dtype=f32, device=dev)
        self.P1 = torch.zeros(self.BP // 16 * self.C.mlpg_p1_floats(), dtype=f32, device=dev)
        self.P2 = torch.zeros(self.nchunk * self.C.mlpg_p2_floats(), dtype=f32, device=dev)
        self.grads = torch.zeros(NPARAM, dtype=f32, device=dev) if self.world_size > 1 else None
        self.lr = torch.tensor([lr], dtype=f32, device=dev)
        self.ring = int(metrics_ring)
        self.metrics = torch.zeros(self.ring * 2, dtype=f32, device=dev)
        self.gstep = torch.zeros(1, dtype=torch.int64, device=dev)
        self.allreduce = "none"
        if self.world_size > 1:
            coll = world.gpu_coll(NPARAM * 4)    # collective: IPC on one node, else RCCL; None on gloo worlds
            self.allreduce = "ipc" if (coll is not None and coll is world.ipc) else \
                ("rccl" if world.comm is not None else world.backend)
        # RCCL and the IPC collectives capture into hipGraphs (the IPC sequence
        # numbers live on the device); a gloo all-reduce does not
        self.graph_safe = self.world_size == 1 or self.allreduce in ("rccl", "ipc")
        self.ipc_parity = 0
        self.shadows_stale = False
        self.set_params(init_params(seed))

    def ipc_error(self) -> int:
        return 0

    def _apply(self, mode: int, gin=None, gout=None, scale: float = 1.0):
        self.C.mlpg_apply(self.params, self.P1, self.P2, self.nchunk, gin, gout, self.lr, scale, self.W1S,
                          self.metrics, self.gstep, self.B, mode)

    def set_params(self, flat_cpu: torch.Tensor, broadcast: bool = True):
        self.params.copy_(flat_cpu.to(self.device, torch.float32))
        if broadcast and self.world is not None and self.world_size > 1:
            self.world.broadcast(self.params, 0)
        self.refresh_shadows()

    def refresh_shadows(self):
        self._apply(3)

    def get_params(self) -> torch.Tensor:
        return self.params.detach().cpu()

    def set_lr(self, lr: float):
        self.lr.fill_(lr)

    @property
    def global_step(self) -> int:
        return int(self.gstep.item())

    def set_global_step(self, v: int):
        self.gstep.fill_(int(v))

    def read_metrics(self, first_step: int, last_step: int) -> np.ndarray:
        m = self.metrics.view(self.ring, 2).cpu().numpy()
        return m[np.arange(first_step, last_step) % self.ring]

    def enqueue_step(self, x: torch.Tensor, x_off: int, x_kind: int, labels: torch.Tensor,
                     labels_off: int, ipc_parity: Optional[int] = None):
        """x: u8 stage holding B rows of 784 pixels at byte offset x_off; labels: u8 class ids."""
        if x_kind != 0:
            raise ValueError("GemmMLPTrainer reads uint8 pixel records (x_kind 0)")
        C, B = self.C, self.B
        C.mlpg_fwd(x, x_off, labels, labels_off, B, self.W1S, self.params, self.a2, self.P1, self.dz2S, self.act,
                   self.naive, 1.0 / B)
        C.mlpg_wgrad(x, x_off, B, self.dz2S, self.P2, self.nchunk)
        if self.world_size == 1:
            self._apply(0)
        else:
            self._apply(1, gout=self.grads)
            self.world.all_reduce(self.grads, "sum")
            self._apply(2, gin=self.grads, scale=1.0 / self.world_size)

    def step_tensors(self, x: torch.Tensor, labels: torch.Tensor):
        """Eager step on device tensors (x: uint8 [B,784], labels [B])."""
        if x.dtype != torch.uint8:
            raise ValueError("GemmMLPTrainer.step_tensors takes uint8 pixels")
        self.enqueue_step(x.contiguous().view(-1), 0, 0, labels.to(torch.uint8).contiguous(), 0)


class MLPStepRunner:
    """Drives `FusedMLPTrainer` over a pinned-host epoch.

    The epoch lives batch-major in pinned host memory; the device holds only a
    *chunk* stage of `g` batches (g*78.5 KB at B=100).  Each chunk is one
    hipGraph: hipMemcpyAsync(chunk, pinned -> stage) followed by the `g` fused
    steps; the host issues one launch per `g` steps.

    prefetch="serial" (default): the copy is a node at the head of the chunk
        graph on the compute stream (+1.7 us/step amortised: 85 us per 3.9 MB
        chunk at PCIe rate).
    prefetch="side": double-buffered stage, the next chunk is copied on a side
        stream under the current replay, synchronised by events.  On MI355X /
        ROCm 7 every cross-queue event dependency costs ~150 us of GPU idle
        (measured, scripts/probes/diag_mlp3.py: 14.9 us/step vs 13.2 serial; the same
        fork/join captured inside the graph: 16.4), so it only pays where
        cross-queue waits are cheap.
    """

    def __init__(self, trainer: FusedMLPTrainer, epoch, steps_per_graph: int = 50,
                 use_graph: bool = True, prefetch: str = "serial"):
        if prefetch not in ("serial", "side"):
            raise ValueError("prefetch must be 'serial' or 'side'")
        self.t = trainer
        self.epoch = epoch
        # a chunk may run across the epoch boundary (its records are copied in two
        # pieces): at large batch an epoch is only ~13 steps, and the side-stream
        # prefetch pays its cross-queue synchronisation once per chunk
        self.g = int(max(1, steps_per_graph))
        self.use_graph = use_graph
        self.prefetch = prefetch
        self.side = torch.cuda.Stream(device=trainer.device)
        self.graphs: Dict[tuple, torch.cuda.CUDAGraph] = {}
        nbuf = 2 if prefetch == "side" else 1
        self.stage = [torch.zeros(self.g * epoch.rec, dtype=torch.uint8, device=trainer.device)
                      for _ in range(nbuf)]
        self.cursor = 0        # next batch index (global)
        self.parity = 0        # (side) stage buffer holding the chunk at `cursor`
        self.loaded = None     # (side) (b0, g) resident in stage[parity]
        self._freed = None     # (side) event: last replay reading stage[parity ^ 1] done

    def _copy_chunk(self, dst: torch.Tensor, b0: int, g: int):
        ep = self.epoch
        nb, off = ep.num_batches, 0
        while g > 0:   # batches b0 .. b0+g-1 of the epoch, wrapping at its end
            n = min(g, nb - b0)
            self.t.C.memcpy_h2d_async(dst, off, ep.host, b0 * ep.rec, n * ep.rec)
            off += n * ep.rec
            b0 = (b0 + n) % nb
            g -= n

    def _emit_steps(self, g: int, buf: torch.Tensor, ipar: int):
        t = self.t
        rec, B = self.epoch.rec, t.B
        for i in range(g):
            off = i * rec
            t.enqueue_step(buf, off, 0, buf, off + B * D_IN, ipc_parity=(ipar + i) & 1)

    def _emit(self, key):
        if self.prefetch == "serial":
            b0, g, ipar = key
            self._copy_chunk(self.stage[0], b0, g)
            self._emit_steps(g, self.stage[0], ipar)
        else:
            g, par, ipar = key
            self._emit_steps(g, self.stage[par], ipar)

    def _graph(self, key) -> torch.cuda.CUDAGraph:
        gr = self.graphs.get(key)
        if gr is None:
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream(device=self.t.device)
            with torch.cuda.graph(gr, stream=s):
                self._emit(key)
            torch.cuda.synchronize()
            self.graphs[key] = gr
        return gr

    def _chunks(self, cursor: int, steps: int) -> List[Tuple[int, int]]:
        out, left = [], steps
        nb = self.epoch.num_batches
        while left > 0:
            b0 = cursor % nb
            g = min(self.g, left)
            out.append((b0, g))
            cursor += g
            left -= g
        return out

    def plan(self, steps: int):
        """[(b0, g, parity, next, ipc_parity)] for the next `steps` steps from the cursor."""
        ch = self._chunks(self.cursor, steps)
        after = self._chunks(self.cursor + steps, self.g)[0]  # speculative prefetch
        out, par, ipar = [], self.parity, self.t.ipc_parity
        for j, (b0, g) in enumerate(ch):
            nxt = ch[j + 1] if j + 1 < len(ch) else after
            out.append((b0, g, par, nxt, ipar))
            par ^= 1
            ipar = (ipar + g) & 1
        return out

    def _key(self, b0, g, par, ipar=0):
        return (b0, g, ipar) if self.prefetch == "serial" else (g, par, ipar)

    def prepare(self, steps: int):
        """Capture every graph `run(steps)` will need (keeps capture out of timing)."""
        if self.use_graph:
            for (b0, g, par, _, ipar) in self.plan(steps):
                self._graph(self._key(b0, g, par, ipar))

    def run(self, steps: int, events: Optional[list] = None):
        main = torch.cuda.current_stream()
        for (b0, g, par, nxt, ipar) in self.plan(steps):
            key = self._key(b0, g, par, ipar)
            self.t.ipc_parity = (ipar + g) & 1
            if self.prefetch == "side" and self.loaded != (b0, g):  # cold start / plan change
                self._copy_chunk(self.stage[par], b0, g)
                self._freed = None
            if self.use_graph:
                self._graph(key).replay()
            else:
                self._emit(key)
            if events is not None:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(main)
                events.append((ev, g))
            if self.prefetch == "side":
                # next chunk into the other buffer, behind the end of the replay that
                # last read it; fresh events (no re-record with pending waits)
                ev_copy = torch.cuda.Event()
                if self._freed is not None:
                    self.side.wait_event(self._freed)
                with torch.cuda.stream(self.side):
                    self._copy_chunk(self.stage[par ^ 1], nxt[0], nxt[1])
                ev_copy.record(self.side)
                self._freed = torch.cuda.Event()
                self._freed.record(main)
                main.wait_event(ev_copy)
                self.parity = par ^ 1
                self.loaded = nxt
            self.cursor += g


class PersistentMLPRunner:
    """Drives a persistent weight-stationary training kernel over a pinned-host
    epoch: ONE launch per chunk of up to `g` steps.

    precision="fp32" (default, the reference's precision: example.py:77-118 is
        fp32 end to end) -- csrc/kernels/mlp_persist_f32.hip, SPLIT: 28 compute
        workgroups (7 hidden blocks x 4 feature slices, packed on one XCD); the
        two big GEMMs (x W1 and x^T dz2) on 16x16x32 bf16 MFMA through the EXACT
        3-way split of their fp32 operand (hi + mid + lo == the fp32 value;
        pixels exact in bf16), so every product is exact and accumulates in
        fp32; the head on f32-input MFMA; fp32 master weights in VGPRs.  Each
        step's x slice is staged into LDS by one wave with LDS-DMA.
    precision="fp32-mfma" -- the same engine with every product on f32-input
        MFMA (v_mfma_f32_16x16x4_f32, bitwise an fmaf chain): 1/8 of the bf16
        MFMA rate, ~2 us/step slower.
    (Rounds 1-3 also carried a 7-workgroup split engine -- one hand-off per
    step but 7 CUs of MFMA work: 14.5 us/step -- and an fp16 engine; both were
    retired in round 4: profiles/README.md.)

    Inside each launch the copier workgroups pull the NEXT chunk from pinned host
    memory over PCIe into the other device stage while the compute workgroups
    run this one.  No second stream, no cross-queue events, no graph capture.

    Staging is range-based: a request whose steps lie inside a staged chunk
    runs from it at an offset (no copy).  The chunk prefetched inside a launch
    is the next planned chunk, or -- for the last launch of a `run()` -- a
    speculative chunk of the same length as that `run()` (`lookahead` overrides
    it, e.g. a warmup priming exactly the timed run), so a short timed run never
    streams more than it computes.  `copy_only_launches` counts cold starts.

    N GPUs of one node (world_size > 1): every compute workgroup exchanges its
    gradient with the same workgroup on every peer through IPC-mapped uncached
    buffers inside the same launch (flag per workgroup and step, rank-order sums
    -> bit-identical replicas).  Batch <= 112 per GPU.

    `step_ts` (int64 ring on the device) receives the s_memrealtime (100 MHz)
    stamp of every global step's start, plus the end of each launch:
    `step_times_ms(first, last)` gives true per-step durations.
    """

    TS_RING = 16384

    def __init__(self, trainer: FusedMLPTrainer, epoch, steps_per_launch: int = 550,
                 timeout_s: float = 30.0, precision: str = "fp32", grad_bf16: bool = True,
                 placement: str = "auto", exchange: str = "one-shot"):
        C = trainer.C
        if precision not in ("fp32", "fp32-mfma"):
            raise ValueError("precision must be 'fp32' or 'fp32-mfma'")
        self.precision = precision
        self.f32 = True
        self.mfma_split = precision == "fp32"
        if exchange not in ("one-shot", "two-shot"):
            raise ValueError("exchange must be 'one-shot' or 'two-shot'")
        # N GPUs: one-shot = each workgroup reads its gradient slot from every
        # peer ((W-1) slots per GPU per step); two-shot = reduce-scatter by wave
        # chunk + all-gather of the sums (2 (W-1)/W of a slot, one more hop)
        self.exchange = exchange
        maxb = C.mlpf_max_batch()
        if trainer.B > maxb:
            raise ValueError(f"PersistentMLPRunner needs batch <= {maxb}")
        if epoch.batch_size != trainer.B:
            raise ValueError("epoch batch size != trainer batch size")
        self.t = trainer
        self.epoch = epoch
        self.g = int(min(steps_per_launch, epoch.num_batches))
        self.timeout_s = float(timeout_s)
        self.grad_bf16 = bool(grad_bf16)
        if placement == "auto":
            # several ranks sharing one GPU (tests): their compute workgroups cannot all sit on one XCD
            nloc = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
            placement = "spread" if nloc > max(1, torch.cuda.device_count()) else "packed"
        if placement not in ("packed", "spread"):
            raise ValueError("placement must be 'auto', 'packed' or 'spread'")
        self.placement = placement
        dev = trainer.device
        self.rec_s = int(C.mlpf_stage_rec())
        self.stages = [torch.zeros(self.g * self.rec_s, dtype=torch.uint8, device=dev) for _ in range(2)]
        self.xbuf = torch.zeros(int(C.mlpf_xbuf_bytes()), dtype=torch.uint8, device=dev)
        self.seq = torch.zeros(1, dtype=torch.int64, device=dev)
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        self.step_ts = torch.zeros(self.TS_RING, dtype=torch.int64, device=dev)
        self.phase_ts = None    # fp32 engine: optional [64 steps][64 wg][16] phase stamps (profiling)
        self._plan = None       # fp32 engine: prepared C++ launcher (PersistF32Plan)
        self.cursor = 0
        self.staged: List[Optional[Tuple[int, int]]] = [None, None]   # (b0, g) resident per stage buffer
        self.copy_only_launches = 0
        self.last_prefetch_steps = 0
        self.use_graph = False  # MLPStepRunner interface
        self.prefetch = "in-kernel"
        self.ipc = None
        self.W, self.rank = 1, 0
        w = trainer.world
        if w is not None and w.world_size > 1:
            if int(os.environ.get("LOCAL_WORLD_SIZE", w.world_size)) != w.world_size:
                raise RuntimeError("the persistent N-GPU exchange needs all ranks on one node")
            from ..parallel.world import open_peer_buffers
            self.ipc = open_peer_buffers(C, int(C.mlpf_ipc_bytes()), w)
            self.W, self.rank = w.world_size, w.rank

    def _chunks(self, cursor: int, steps: int) -> List[Tuple[int, int]]:
        out, left = [], steps
        nb = self.epoch.num_batches
        while left > 0:
            b0 = cursor % nb
            g = min(self.g, left, nb - b0)
            out.append((b0, g))
            cursor += g
            left -= g
        return out

    def _launch(self, par: int, off: int, nsteps: int, nxt: Tuple[int, int]):
        """Run `nsteps` from stage `par` at step offset `off`; copy `nxt` into stage par^1."""
        t, ep = self.t, self.epoch
        dst = par ^ 1
        ipc = dict(ipc_table=self.ipc.table_ptr() if self.ipc is not None else 0, ipc_W=self.W, ipc_rank=self.rank)
        if self.phase_ts is None:
            if self._plan is None:   # every pointer resolved once (host-side launch cost)
                self._plan = t.C.PersistF32Plan(
                    self.stages[0], self.stages[1], ep.rec, t.B, t.params, t.lr, t.metrics, t.gstep, self.seq,
                    self.xbuf, self.err, self.timeout_s, t.act, int(t.naive), ep.host, self.step_ts,
                    ipc["ipc_table"], self.W, self.rank, self.grad_bf16, self.placement == "spread",
                    self.exchange == "two-shot", self.mfma_split)
            self._plan.launch(par, off if nsteps > 0 else 0, nsteps, nxt[0] * ep.rec, nxt[1])
        else:   # phase stamps (profiling): the generic binding
            st = self.stages[par][off * self.rec_s:] if nsteps > 0 else self.stages[par]
            t.C.mlp_persist_f32(st, ep.rec, t.B, nsteps, t.params, t.lr, t.metrics, t.gstep, self.seq, self.xbuf,
                                self.err, self.timeout_s, t.act, int(t.naive), host=ep.host,
                                host_offset=nxt[0] * ep.rec, next_steps=nxt[1], stage_next=self.stages[dst],
                                step_ts=self.step_ts, grad_bf16=self.grad_bf16, phase_ts=self.phase_ts,
                                spread=self.placement == "spread", two_shot=self.exchange == "two-shot",
                                mfma_split=self.mfma_split, **ipc)
        if nxt[1] > 0:
            self.staged[dst] = nxt
        self.last_prefetch_steps = nxt[1]

    def _locate(self, b0: int, g: int) -> Optional[Tuple[int, int]]:
        for par in (0, 1):
            s = self.staged[par]
            if s is not None and s[0] <= b0 and b0 + g <= s[0] + s[1]:
                return par, b0 - s[0]
        return None

    def _ensure(self, b0: int, g: int) -> Tuple[int, int]:
        """(stage, offset) holding steps [b0, b0+g); copy-only launch on a miss."""
        loc = self._locate(b0, g)
        if loc is None:
            # cold start / plan change: copy (b0, g) into a stage buffer with a
            # copy-only launch (the stage it "runs" from is untouched)
            dst = 0 if self.staged[0] is None else (1 if self.staged[1] is None else 0)
            par = dst ^ 1
            self._launch(par, 0, 0, (b0, g))
            self.copy_only_launches += 1
            loc = (par ^ 1, 0)
        return loc

    def prepare(self, steps: int):
        """Stage the first chunk of the next `run(steps)` (outside any timed region)."""
        b0, g = self._chunks(self.cursor, steps)[0]
        self._ensure(b0, g)

    def invalidate(self):
        """Forget staged chunks (call after re-packing the pinned epoch, e.g. a shuffle)."""
        self.staged = [None, None]

    def error(self) -> int:
        return int(self.err.item())

    def run(self, steps: int, events: Optional[list] = None, lookahead: Optional[int] = None):
        if events is None and self._plan is not None and self._run_fast(steps, lookahead):
            return
        main = torch.cuda.current_stream()
        ch = self._chunks(self.cursor, steps)
        la = min(self.g, steps if lookahead is None else int(lookahead))
        for k, (b0, g) in enumerate(ch):
            if k + 1 < len(ch):
                nxt = ch[k + 1]
            else:
                nxt = self._chunks(self.cursor + g, la)[0] if la > 0 else (0, 0)
            par, off = self._ensure(b0, g)
            if nxt[1] > 0 and self.staged[par ^ 1] is not None and self._covers(self.staged[par ^ 1], nxt):
                nxt_copy = (nxt[0], 0)      # already resident in the other stage: nothing to stream
            else:
                nxt_copy = nxt
            self._launch(par, off, g, nxt_copy)
            if events is not None:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(main)
                events.append((ev, g))
            self.cursor += g
        self.t.shadows_stale = True

    def _run_fast(self, steps: int, lookahead: Optional[int]) -> bool:
        """run() for the common case -- one chunk, already staged, the resolved
        launch plan -- with the least host work in front of the launch (the
        host call is inside a short timed run: ~14 us through the general path).
        Same launch and bookkeeping as the general path; False when it does not apply."""
        nb = self.epoch.num_batches
        b0 = self.cursor % nb
        if steps <= 0 or steps > self.g or b0 + steps > nb or self.phase_ts is not None:
            return False
        s0, s1 = self.staged
        if s0 is not None and s0[0] <= b0 and b0 + steps <= s0[0] + s0[1]:
            par, off = 0, b0 - s0[0]
        elif s1 is not None and s1[0] <= b0 and b0 + steps <= s1[0] + s1[1]:
            par, off = 1, b0 - s1[0]
        else:
            return False
        la = min(self.g, steps if lookahead is None else int(lookahead))
        nxt = (0, 0)
        if la > 0:
            c = (self.cursor + steps) % nb
            nxt = (c, min(self.g, la, nb - c))
            o = self.staged[par ^ 1]
            if o is not None and o[0] <= nxt[0] and nxt[0] + nxt[1] <= o[0] + o[1]:
                nxt = (nxt[0], 0)             # already resident in the other stage
        rec = self.epoch.rec
        self._plan.launch(par, off, steps, nxt[0] * rec, nxt[1])
        if nxt[1] > 0:
            self.staged[par ^ 1] = nxt
        self.last_prefetch_steps = nxt[1]
        self.cursor += steps
        self.t.shadows_stale = True
        return True

    @staticmethod
    def _covers(s: Tuple[int, int], r: Tuple[int, int]) -> bool:
        return s[0] <= r[0] and r[0] + r[1] <= s[0] + s[1]

    def step_times_ms(self, first: int, last: int) -> np.ndarray:
        """Per-step durations (ms) of global steps [first, last) from the device stamps."""
        if last - first >= self.TS_RING:
            first = last - self.TS_RING + 1
        ts = self.step_ts.cpu().numpy()
        idx = np.arange(first, last + 1) % self.TS_RING
        return np.diff(ts[idx]).astype(np.float64) * 1e-5     # 100 MHz ticks -> ms
