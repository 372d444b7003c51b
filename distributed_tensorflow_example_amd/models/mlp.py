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
                 metrics_ring: int = 8192, seed: int = 1, device=None):
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
        self.xT = torch.zeros(800 * self.BP, dtype=bf, device=dev)
        self.dz2T = torch.zeros(112 * self.BP, dtype=bf, device=dev)
        self.partials = torch.zeros(self.nb * 1112, dtype=torch.float32, device=dev)
        self.grad_dtype = grad_dtype
        self.grads = (torch.zeros(NPARAM, dtype=grad_dtype, device=dev)
                      if self.world_size > 1 else None)
        self.lr = torch.tensor([lr], dtype=torch.float32, device=dev)
        self.ring = int(metrics_ring)
        self.metrics = torch.zeros(self.ring * 2, dtype=torch.float32, device=dev)
        self.gstep = torch.zeros(1, dtype=torch.int64, device=dev)
        from ..data.mnist import record_bytes

        self.rec = record_bytes(B)
        self.slots = [torch.zeros(self.rec, dtype=torch.uint8, device=dev) for _ in range(2)]
        self.set_params(init_params(seed))

    # ---------------------------------------------------------------- state
    def set_params(self, flat_cpu: torch.Tensor, broadcast: bool = True):
        self.params.copy_(flat_cpu.to(self.device, torch.float32))
        if broadcast and self.world is not None and self.world_size > 1:
            self.world.broadcast(self.params, 0)  # chief init + broadcast
        self.refresh_shadows()

    def refresh_shadows(self):
        self.C.mlp_apply_flat(self.params, None, self.lr, 0.0, self.W1T, self.W2T)

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
    def compute(self, slot: torch.Tensor):
        """Enqueue one training step reading batch record `slot` (device)."""
        C = self.C
        B = self.B
        C.mlp_fwd_bwd(slot, 0, 0, slot, B * D_IN, B, self.W1T, self.W2T, self.params, self.xT,
                      self.dz2T, self.BP, self.partials, 1.0 / B, self.act, self.naive)
        self.after_fwd_bwd()

    def after_fwd_bwd(self):
        C = self.C
        if self.world_size == 1:
            C.mlp_wgrad(self.xT, self.dz2T, self.BP, self.B, self.partials, self.params, self.W1T,
                        self.W2T, None, 0, self.lr, self.metrics, self.gstep)
        else:
            kind = 1 if self.grad_dtype == torch.float32 else 2
            C.mlp_wgrad(self.xT, self.dz2T, self.BP, self.B, self.partials, self.params, self.W1T,
                        self.W2T, self.grads, kind, self.lr, self.metrics, self.gstep)
            self.world.comm.all_reduce(self.grads, "sum")
            C.mlp_apply_flat(self.params, self.grads, self.lr, 1.0 / self.world_size, self.W1T,
                             self.W2T)

    def step_tensors(self, x: torch.Tensor, labels: torch.Tensor):
        """Eager step on device tensors (x: uint8/fp32/bf16 [B,784], labels uint8 [B])."""
        kind = {torch.uint8: 0, torch.float32: 1, torch.bfloat16: 2}[x.dtype]
        x = x.contiguous()
        lab = labels.to(torch.uint8).contiguous()
        self.C.mlp_fwd_bwd(x, 0, kind, lab, 0, self.B, self.W1T, self.W2T, self.params, self.xT,
                           self.dz2T, self.BP, self.partials, 1.0 / self.B, self.act, self.naive)
        self.after_fwd_bwd()


class MLPStepRunner:
    """Drives `FusedMLPTrainer` over a pinned-host epoch.

    Per step: side stream -- hipMemcpyAsync of batch i+1 (pinned -> device
    double buffer) once step i-1 has consumed that slot; main stream -- wait
    for batch i, fwd/bwd kernel, wgrad(+SGD | all-reduce + apply).  `g` such
    steps are captured into one hipGraph (keyed by first batch index) and
    replayed, so the host issues one launch per `g` steps.
    """

    def __init__(self, trainer: FusedMLPTrainer, epoch, steps_per_graph: int = 50,
                 use_graph: bool = True):
        self.t = trainer
        self.epoch = epoch
        self.g = int(steps_per_graph)
        self.use_graph = use_graph
        self.side = torch.cuda.Stream(device=trainer.device)
        self.graphs: Dict[Tuple[int, int], torch.cuda.CUDAGraph] = {}
        self.cursor = 0  # next batch index (global, mod num_batches)

    def _emit(self, b0: int, g: int):
        t, C, ep = self.t, self.t.C, self.epoch
        main = torch.cuda.current_stream()
        side = self.side
        start = torch.cuda.Event()
        start.record(main)
        copied = [torch.cuda.Event() for _ in range(g)]
        consumed = [torch.cuda.Event() for _ in range(g)]
        nbytes = ep.rec

        def copy(i):
            b = (b0 + i) % ep.num_batches
            C.memcpy_h2d_async(t.slots[i % 2], 0, ep.host, b * ep.rec, nbytes)

        with torch.cuda.stream(side):
            side.wait_event(start)
            copy(0)
            copied[0].record(side)
        for i in range(g):
            if i + 1 < g:
                with torch.cuda.stream(side):
                    if i >= 1:
                        side.wait_event(consumed[i - 1])
                    copy(i + 1)
                    copied[i + 1].record(side)
            main.wait_event(copied[i])
            slot = t.slots[i % 2]
            B = t.B
            C.mlp_fwd_bwd(slot, 0, 0, slot, B * D_IN, B, t.W1T, t.W2T, t.params, t.xT, t.dz2T,
                          t.BP, t.partials, 1.0 / B, t.act, t.naive)
            consumed[i].record(main)
            t.after_fwd_bwd()

    def _graph(self, b0: int, g: int) -> torch.cuda.CUDAGraph:
        key = (b0, g)
        gr = self.graphs.get(key)
        if gr is None:
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream(device=self.t.device)
            with torch.cuda.graph(gr, stream=s):
                self._emit(b0, g)
            torch.cuda.synchronize()
            self.graphs[key] = gr
        return gr

    def plan(self, steps: int) -> List[Tuple[int, int]]:
        out, cur, left = [], self.cursor, steps
        nb = self.epoch.num_batches
        while left > 0:
            b0 = cur % nb
            g = min(self.g, left, nb - b0)
            out.append((b0, g))
            cur += g
            left -= g
        return out

    def prepare(self, steps: int):
        """Capture every graph `run(steps)` will need (keeps capture out of timing)."""
        if self.use_graph:
            for b0, g in self.plan(steps):
                self._graph(b0, g)

    def run(self, steps: int, events: Optional[list] = None):
        for b0, g in self.plan(steps):
            if self.use_graph:
                self._graph(b0, g).replay()
            else:
                self._emit(b0, g)
            if events is not None:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                events.append((ev, g))
            self.cursor += g
