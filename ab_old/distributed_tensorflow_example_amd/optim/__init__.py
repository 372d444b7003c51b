"""Fused multi-tensor optimizers (csrc/kernels/ops.hip: multi_tensor_apply).

One launch updates every parameter of a group: the
reference's per-variable ApplyGradientDescent / ApplyAdam ops become a single
kernel over a (tensor, 4096-element chunk) work list.  Learning rate and step
live on the device so a whole training step (including the update) can be
captured in a hipGraph and the schedule changed without re-capture.

Semantics follow TensorFlow where the reference uses it:
  GradientDescent  p -= lr * g                         (example.py:108)
  Momentum         m = mu*m + g; p -= lr*m (or Nesterov)
  Adam (TF)        lr_t = lr*sqrt(1-b2^t)/(1-b1^t); p -= lr_t*m/(sqrt(v)+eps)
                   (epsilon outside the sqrt, "epsilon hat"; model_export.py:38)
  AdamW            decoupled weight decay (BERT recipe)
  Adagrad (TF)     acc += g^2; p -= lr*g/sqrt(acc)      (acc starts at 0.1)
  RMSProp (TF)     ms = rho*ms + (1-rho)*g^2; mom = mu*mom + lr*g/sqrt(ms+eps); p -= mom
                   (ms starts at 1, as TF's RMSPropOptimizer initialises it)
`grad_scale` folds the 1/N of a summed all-reduce into the update.
CPU tensors use the same math in PyTorch (CPU/gloo configuration).
"""
from __future__ import annotations

from typing import Iterable, List, Optional

import torch

from .. import _native

_bump_version = torch.autograd.graph.increment_version

KINDS = {"sgd": 0, "momentum": 1, "adam": 2, "adamw": 3, "adagrad": 4, "rmsprop": 5}


_F32_TINY = 1.1754943508222875e-38   # smallest normal float32
_F32_ZERO_BELOW = 2.0 ** -150         # a float32 power this small rounds to 0.0


def adam_steps_from_powers(beta1_power: Optional[float], beta1: float,
                           beta2_power: Optional[float] = None, beta2: Optional[float] = None) -> int:
    """Adam's update count t from TF's saved non-slot accumulators beta^(t+1).

    The powers are float32: beta1 = 0.9 turns subnormal near t = 830 and 0.0
    near t = 990; beta2 = 0.999 stays normal to t ~ 87,000 and reaches 0.0
    near t ~ 103,000.  The step comes from whichever power is still a normal
    float (those are exact to far below one step); a subnormal power is too
    coarse and only bounds t from below.  When every power has underflowed the
    bias correction is 1 to float precision (TF keeps the power at 0), so the
    count saturates at the first step where every power is 0.0 -- never at 0,
    which would restart the bias correction (lr ~0.3x for thousands of steps)."""
    import math

    best, bound = None, 0
    for v, beta in ((beta1_power, beta1), (beta2_power, beta2)):
        if v is None or beta is None or not (0.0 < beta < 1.0):
            continue
        v = float(v)
        if _F32_TINY <= v < 1.0:
            best = max(0, int(round(math.log(v) / math.log(beta))) - 1)
            break
        if 0.0 < v < _F32_TINY:       # subnormal: t + 1 >= log(tiny) / log(beta)
            bound = max(bound, int(math.floor(math.log(v) / math.log(beta))) - 1)
        elif v <= 0.0:                # underflowed: t + 1 > log(2^-150) / log(beta)
            bound = max(bound, int(math.ceil(math.log(_F32_ZERO_BELOW) / math.log(beta))))
    if best is not None:
        return best
    return max(0, bound)


def _dense(t: torch.Tensor) -> bool:
    """Non-overlapping dense storage (row-major or channels_last): the kernels
    walk params/grads/slots as flat arrays, so only identical layouts matter."""
    return t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last))


def _same_layout(a: torch.Tensor, b: torch.Tensor) -> bool:
    # strides of size-1 dims are irrelevant (a [o, i, 1, 1] weight is both contiguous and channels_last)
    return a.shape == b.shape and all(x == y for x, y, n in zip(a.stride(), b.stride(), a.shape) if n > 1)


class _FusedBase:
    kind = "sgd"

    def __init__(self, params: Iterable[torch.nn.Parameter], lr: float, weight_decay: float = 0.0,
                 beta1: float = 0.9, beta2: float = 0.999, eps: float = 1e-8, momentum: float = 0.0,
                 nesterov: bool = False):
        self.params: List[torch.Tensor] = [p for p in params]
        if not self.params:
            raise ValueError("optimizer got an empty parameter list")
        self.device = self.params[0].device
        self.wd, self.b1, self.b2, self.eps = weight_decay, beta1, beta2, eps
        self.momentum, self.nesterov = momentum, nesterov
        self.lr_t = torch.tensor([float(lr)], dtype=torch.float32, device=self.device)
        self.step_t = torch.zeros(1, dtype=torch.int64, device=self.device)
        need_m = self.kind in ("momentum", "adam", "adamw", "adagrad", "rmsprop")
        need_v = self.kind in ("adam", "adamw", "rmsprop")
        m0 = {"adagrad": self._init_acc(), "rmsprop": 1.0}.get(self.kind, 0.0)
        self.m = [torch.full_like(p, m0, dtype=torch.float32) if need_m else None for p in self.params]
        self.v = [torch.zeros_like(p, dtype=torch.float32) if need_v else None for p in self.params]
        self._tab_key = None
        self._tab = None
        self._chunks = None
        self.shadows = {}

    def attach_shadow(self, param: torch.Tensor, shadow: torch.Tensor):
        """Keep `shadow` (bf16, same layout) equal to bf16(param) after every step,
        written by the optimizer kernel itself -- no separate cast kernels."""
        if shadow.dtype != torch.bfloat16 or shadow.shape != param.shape or not _same_layout(param, shadow):
            raise ValueError("shadow must be a bf16 tensor with the param's shape and layout")
        self.shadows[id(param)] = shadow
        with torch.no_grad():
            shadow.copy_(param)
        self._tab_key = None

    def _init_acc(self) -> float:
        return 0.0

    # ------------------------------------------------------------------ state
    @property
    def lr(self) -> float:
        return float(self.lr_t.item())

    def set_lr(self, lr: float):
        self.lr_t.fill_(float(lr))

    def state_dict(self):
        return {"lr": self.lr, "step": int(self.step_t.item()),
                "m": [t.detach().cpu() if t is not None else None for t in self.m],
                "v": [t.detach().cpu() if t is not None else None for t in self.v]}

    def load_state_dict(self, sd):
        self.set_lr(sd["lr"])
        self.step_t.fill_(int(sd["step"]))
        for dst, src in zip(self.m, sd["m"]):
            if dst is not None and src is not None:
                dst.copy_(src)
        for dst, src in zip(self.v, sd["v"]):
            if dst is not None and src is not None:
                dst.copy_(src)

    def zero_grad(self, set_to_none: bool = False):
        for p in self.params:
            if p.grad is not None:
                if set_to_none:
                    p.grad = None
                else:
                    p.grad.zero_()

    # ------------------------------------------------------------------ native table
    def _table(self, grads):
        key = tuple((p.data_ptr(), g.data_ptr(), g.dtype) for p, g in zip(self.params, grads))
        if key != self._tab_key:
            C = _native.load()
            chunk = C.mt_chunk()
            rows, chunks = [], []
            for i, (p, g) in enumerate(zip(self.params, grads)):
                if p.dtype != torch.float32 or not _dense(p) or not _same_layout(p, g) or not _dense(g):
                    raise ValueError("fused optimizer needs dense fp32 params with grads of identical layout")
                m, v = self.m[i], self.v[i]
                sh = self.shadows.get(id(p))
                rows.append([p.data_ptr(), g.data_ptr(), m.data_ptr() if m is not None else 0,
                             v.data_ptr() if v is not None else 0, p.numel(),
                             sh.data_ptr() if sh is not None else 0])
                for s in range(0, p.numel(), chunk):
                    chunks.append([i, s])
            self._tab = torch.tensor(rows, dtype=torch.int64).to(self.device)
            self._chunks = torch.tensor(chunks, dtype=torch.int32).reshape(-1, 2).to(self.device)
            self._tab_key = key
        return self._tab, self._chunks

    def _grads(self, grads):
        if grads is None:
            grads = [p.grad for p in self.params]
        out = []
        for p, g in zip(self.params, grads):
            out.append(torch.zeros_like(p) if g is None else g)
        return out

    @torch.no_grad()
    def step(self, grads: Optional[List[torch.Tensor]] = None, grad_scale: float = 1.0,
             skip: Optional[torch.Tensor] = None):
        """One fused update.  `skip`: optional device int32 [1] flag; when it is set
        (a voided step, e.g. a sharded-table exchange overflow) nothing changes --
        no parameter, slot or step count -- decided on the device, no host sync."""
        grads = self._grads(grads)
        if skip is None:
            self.step_t += 1
        else:
            self.step_t += (1 - skip.reshape(-1)[:1]).to(self.step_t.dtype)
        if self.device.type != "cuda":
            if skip is not None and int(skip.reshape(-1)[0]) != 0:
                return None
            return self._step_cpu(grads, grad_scale)
        gdt = {g.dtype for g in grads}
        if len(gdt) != 1 or next(iter(gdt)) not in (torch.float32, torch.bfloat16):
            grads = [g.float() for g in grads]
        gbf = grads[0].dtype == torch.bfloat16
        tab, chunks = self._table(grads)
        _native.load().multi_tensor_apply(tab, chunks, KINDS[self.kind], gbf, self.lr_t, 0.0,
                                          float(grad_scale), self.wd, self.b1, self.b2, self.eps,
                                          self.momentum, self.nesterov, self.step_t,
                                          None if skip is None else skip.reshape(-1)[:1].to(torch.int32))
        # the kernel rewrote the bf16 shadows in place: bump their version counters as
        # an in-place torch op would (caches keyed on them, e.g. ops/conv.py's flipped
        # filters, see the change; a graph still holding an old shadow raises as usual)
        for sh in self.shadows.values():
            _bump_version(sh)

    def _step_cpu(self, grads, gs):
        self._step_cpu_math(grads, gs)
        for p in self.params:
            sh = self.shadows.get(id(p))
            if sh is not None:
                sh.copy_(p)

    def _step_cpu_math(self, grads, gs):
        lr = float(self.lr_t.item())
        t = int(self.step_t.item())
        for i, (p, g) in enumerate(zip(self.params, grads)):
            g = g.float() * gs
            if self.kind == "sgd":
                if self.wd:
                    g = g + self.wd * p
                p.sub_(lr * g)
            elif self.kind == "momentum":
                if self.wd:
                    g = g + self.wd * p
                m = self.m[i]
                m.mul_(self.momentum).add_(g)
                p.sub_(lr * (g + self.momentum * m if self.nesterov else m))
            elif self.kind == "adagrad":
                m = self.m[i]
                m.add_(g * g)
                p.sub_(lr * g / m.sqrt())
            elif self.kind == "rmsprop":
                m, v = self.m[i], self.v[i]
                m.mul_(self.b1).add_((1 - self.b1) * g * g)
                v.mul_(self.momentum).add_(lr * g / (m + self.eps).sqrt())
                p.sub_(v)
            else:
                if self.kind == "adam" and self.wd:
                    g = g + self.wd * p
                m, v = self.m[i], self.v[i]
                m.mul_(self.b1).add_((1 - self.b1) * g)
                v.mul_(self.b2).add_((1 - self.b2) * g * g)
                lr_t = lr * (1 - self.b2 ** t) ** 0.5 / (1 - self.b1 ** t)
                p0 = p.clone() if self.kind == "adamw" else None
                p.sub_(lr_t * m / (v.sqrt() + self.eps))
                if self.kind == "adamw" and self.wd:
                    p.sub_(lr * self.wd * p0)


class FusedSGD(_FusedBase):
    kind = "sgd"

    def __init__(self, params, lr, weight_decay=0.0):
        super().__init__(params, lr, weight_decay=weight_decay)


class FusedMomentum(_FusedBase):
    kind = "momentum"

    def __init__(self, params, lr, momentum=0.9, nesterov=False, weight_decay=0.0):
        super().__init__(params, lr, weight_decay=weight_decay, momentum=momentum, nesterov=nesterov)


class FusedAdam(_FusedBase):
    """TF AdamOptimizer semantics (defaults lr=0.001, b1=0.9, b2=0.999, eps=1e-8)."""

    kind = "adam"

    def __init__(self, params, lr=0.001, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0):
        super().__init__(params, lr, weight_decay=weight_decay, beta1=beta1, beta2=beta2, eps=eps)


class FusedAdamW(_FusedBase):
    kind = "adamw"

    def __init__(self, params, lr=1e-4, beta1=0.9, beta2=0.999, eps=1e-6, weight_decay=0.01):
        super().__init__(params, lr, weight_decay=weight_decay, beta1=beta1, beta2=beta2, eps=eps)


class FusedAdagrad(_FusedBase):
    """TF AdagradOptimizer (initial_accumulator_value 0.1)."""

    kind = "adagrad"

    def __init__(self, params, lr, initial_accumulator_value=0.1):
        self._acc0 = float(initial_accumulator_value)
        super().__init__(params, lr)

    def _init_acc(self) -> float:
        return self._acc0


class FusedRMSProp(_FusedBase):
    """TF RMSPropOptimizer (decay 0.9, momentum 0, epsilon 1e-10; ms slot starts at 1)."""

    kind = "rmsprop"

    def __init__(self, params, lr, decay=0.9, momentum=0.0, epsilon=1e-10):
        super().__init__(params, lr, beta1=decay, eps=epsilon, momentum=momentum)


def global_grad_norm(grads: List[torch.Tensor]) -> torch.Tensor:
    """sqrt(sum g^2) over tensors, one fused launch on GPU."""
    if not grads:
        return torch.zeros(())
    if not grads[0].is_cuda:
        return torch.sqrt(sum((g.float() ** 2).sum() for g in grads))
    C = _native.load()
    chunk = C.mt_chunk()
    rows, chunks = [], []
    for i, g in enumerate(grads):
        g = g.contiguous()
        rows.append([g.data_ptr(), g.data_ptr(), 0, 0, g.numel(), 0])
        for s in range(0, g.numel(), chunk):
            chunks.append([i, s])
    dev = grads[0].device
    tab = torch.tensor(rows, dtype=torch.int64).to(dev)
    ch = torch.tensor(chunks, dtype=torch.int32).reshape(-1, 2).to(dev)
    out = torch.zeros(1, dtype=torch.float32, device=dev)
    C.multi_tensor_sumsq(tab, ch, grads[0].dtype == torch.bfloat16, out)
    return out.sqrt()[0]
