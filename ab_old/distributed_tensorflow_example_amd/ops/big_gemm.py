"""The three products of a bf16 linear layer on the large-tile LDS-DMA MFMA
GEMM (csrc/kernels/gemm_big.hip), with no transpose copies:

    forward        y  = x W^T          (x [T,in], W [out,in])
    input grad     dx = dy W  (+ r)    (beta = 1 folds a residual-branch gradient in)
    weight grad    dW = dy^T x (+= dW) fp32 out, split-K over the T tokens

Shapes outside the kernel's contract (K % 64, 16-byte alignment) go to
torch's GEMM (hipBLASLt).  `use_native(role, M, N, K)` decides per product
which engine a model runs: DTF_BIG_GEMM=auto (default) -- both engines timed
once per shape on scratch operands, the faster one kept -- never (hipBLASLt),
or always (`scripts/bench_gemm.py` prints the same comparison for BERT's shapes).
"""
from __future__ import annotations

import os

import torch

from .. import _native

# auto (default): both engines timed once per shape (best of 3 rounds), the
# faster one kept -- with the 8-phase schedule this kernel is 0.93-1.09x of
# hipBLASLt on BERT-base's forward / input-gradient shapes and 0.82-1.03x on the
# weight gradients (profiles/gemm_8ph_r3.txt); end to end 'auto' measured equal
# to 'never' and 'always' 3 % slower;  never: hipBLASLt;  always: this kernel
_POLICY = os.environ.get("DTF_BIG_GEMM", "auto")
# hysteresis of 'auto': the in-tree kernel keeps a product unless hipBLASLt is
# faster by more than this fraction -- shapes within a few percent used to flip
# with one-time timing noise from box to box, and with them the
# step's kernel mix; the in-tree side also carries the fused epilogues
_MARGIN = float(os.environ.get("DTF_BIG_GEMM_MARGIN", "0.05"))
# fused GELU epilogues: 1 both (use_gelu_aux, use_dgelu), bwd only the backward one, 0 none
_GELU_EPI = os.environ.get("DTF_GEMM_DGELU", "1")
_DGELU = _GELU_EPI != "0"
_GELU_AUX = _GELU_EPI not in ("0", "bwd")
_choice: dict = {}
_timings: dict = {}
# Fixed per-shape engine table for BERT-base at B = 128, S = 128 (T = 16384
# token rows; DTF_BIG_GEMM_TABLE=0: time every shape): the choice set of the
# fastest measured run (8,370-8,393 seq/s, profiles/bert_gemm_margin_ab_r5.txt).
# The one-time timing flips the near-tie products from box to box (FFN2 weight
# gradient, QKV / FFN1 input gradients: in-tree within 5 % on the microbench,
# slower in the step), and the step with them moved ran 7,869-8,096 seq/s
# (profiles/bert_base_b128_r5_*.json).  Shapes not listed are timed.
_TABLE_ON = os.environ.get("DTF_BIG_GEMM_TABLE", "1") != "0"
_TABLE = {
    ("fwd", 16384, 2304, 768): True, ("fwd", 16384, 768, 768): True, ("fwd", 16384, 3072, 768): True,
    ("gelu_aux", 16384, 3072, 768): True, ("dgelu", 16384, 3072, 768): True,
    ("dx", 16384, 768, 768): True, ("dw", 768, 3072, 16384): True, ("dw", 2304, 768, 16384): True,
    ("fwd", 16384, 768, 3072): False, ("dx", 16384, 3072, 768): False, ("dx", 16384, 768, 3072): False,
    ("dx", 16384, 768, 2304): False, ("dw", 3072, 768, 16384): False, ("dw", 768, 768, 16384): False,
}


# A/B runs: DTF_BIG_GEMM_SET="dx:16384:768:3072=1,fwd:16384:768:3072=0" overrides
# single table entries (1 = gemm_big, 0 = hipBLASLt)
_OVERRIDE = {}
for _item in filter(None, os.environ.get("DTF_BIG_GEMM_SET", "").split(",")):
    _k, _v = _item.split("=")
    _r, _m, _n, _kk = _k.split(":")
    _OVERRIDE[(_r, int(_m), int(_n), int(_kk))] = _v.strip() == "1"


def _fixed(key):
    """The table's engine for `key` under 'auto' (None: not listed / table off)."""
    if key in _OVERRIDE:
        return _OVERRIDE[key]
    if not _TABLE_ON or _POLICY != "auto":
        return None
    return _TABLE.get(key)


def _C():
    return _native.load()


def _time(fn, reps=5, rounds=5):
    """Best-of-`rounds` mean time (ms) of `reps` back-to-back calls."""
    fn()
    best = float("inf")
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / reps)
    return best


def policy() -> str:
    return _POLICY


def _candidates(role, M, N, K, dev):
    """(ours, torch) closures for one product on scratch operands of its shape."""
    C = _C()
    bf = torch.bfloat16
    if role == "fwd":      # y[M,N] = x[M,K] W[N,K]^T
        a, b = torch.randn(M, K, device=dev, dtype=bf), torch.randn(N, K, device=dev, dtype=bf)
        o = torch.empty(M, N, device=dev, dtype=bf)
        return (lambda: C.gemm_big(a, False, b, True, o)), (lambda: torch.mm(a, b.t(), out=o))
    if role == "dx":       # dx[M,N] = dy[M,K] W[K,N]
        a, b = torch.randn(M, K, device=dev, dtype=bf), torch.randn(K, N, device=dev, dtype=bf)
        o = torch.empty(M, N, device=dev, dtype=bf)
        return (lambda: C.gemm_big(a, False, b, False, o)), (lambda: torch.mm(a, b, out=o))
    # dw[M,N] += dy[K,M]^T x[K,N]; the torch side is what the models run without
    # this kernel: token-slab batched GEMM + slab_sum (models/bert.py _wgrad)
    a, b = torch.randn(K, M, device=dev, dtype=bf), torch.randn(K, N, device=dev, dtype=bf)
    o = torch.zeros(M, N, device=dev)

    def theirs():
        from ..models.bert import _wgrad_torch
        _wgrad_torch(a, b, into=o)
    return (lambda: C.gemm_big(a, True, b, False, o, beta=1.0, split_k=0)), theirs


def use_native(role: str, M: int, N: int, K: int, dev) -> bool:
    """True when gemm_big should run this product: the policy, the kernel's
    shape contract (K % 64), and -- under 'auto' -- a one-time timing of both
    engines on scratch operands of the shape (cached per process)."""
    if _POLICY == "never" or K % 64 or torch.device(dev).type != "cuda":
        return False
    if _POLICY == "always":
        return True
    key = (role, M, N, K)
    hit = _choice.get(key)
    if hit is None and _fixed(key) is not None:
        hit = _choice[key] = _fixed(key)
    if hit is None:
        if torch.cuda.is_current_stream_capturing():
            return False
        ours, theirs = _candidates(role, M, N, K, dev)
        t_ours, t_theirs = _time(ours), _time(theirs)
        hit = _choice[key] = t_ours <= t_theirs * (1.0 + _MARGIN)
        _timings[key] = (round(t_ours, 4), round(t_theirs, 4))
    return hit


def gelu_bwd_slices(M: int) -> int:
    """Row slices of the standalone bias + GELU backward (ops.transformer)."""
    return max(1, min(512, M // 32))


def use_dgelu(M: int, N: int, K: int, dev) -> bool:
    """True when the input gradient of a linear layer fed by bias + GELU should
    run as ONE gemm_big launch with the GELU backward and the bias-gradient
    partials in its epilogue (gemm_dgelu) instead of the dX GEMM (whichever
    engine use_native picks) + the bias_gelu_bwd pass; timed once per shape
    under 'auto'."""
    if (_POLICY == "never" or not _DGELU or M % 256 or N % 256 or K % 128
            or torch.device(dev).type != "cuda"):
        return False
    if _POLICY == "always":
        return True
    key = ("dgelu", M, N, K)
    hit = _choice.get(key)
    if hit is None and _fixed(key) is not None:
        hit = _choice[key] = _fixed(key)
    if hit is None:
        if torch.cuda.is_current_stream_capturing():
            return False
        C = _C()
        bf = torch.bfloat16
        a, b = torch.randn(M, K, device=dev, dtype=bf), torch.randn(K, N, device=dev, dtype=bf)
        aux, out = torch.randn(M, N, device=dev, dtype=bf), torch.empty(M, N, device=dev, dtype=bf)
        bias, db = torch.randn(N, device=dev), torch.empty(N, device=dev)
        colpart = torch.empty((M // 128) * N, device=dev)
        part = torch.empty(gelu_bwd_slices(M) * N, device=dev)
        if not C.gemm_dgelu(a, False, b, False, out, aux, bias, colpart, db):
            _choice[key] = False
            return False
        native_dx = use_native("dx", M, N, K, dev)

        def theirs():
            dh = linear_dx(a, b) if native_dx else torch.mm(a, b)
            C.bias_gelu_bwd(dh, aux, bias, out, part, db, accumulate=False)
        t_ours = _time(lambda: C.gemm_dgelu(a, False, b, False, out, aux, bias, colpart, db))
        t_theirs = _time(theirs)
        hit = _choice[key] = t_ours <= t_theirs * (1.0 + _MARGIN)
        _timings[key] = (round(t_ours, 4), round(t_theirs, 4))
    return hit


def use_gelu_aux(M: int, N: int, K: int, dev) -> bool:
    """True when the forward of a linear layer followed by bias + GELU should
    run as ONE gemm_big launch writing the pre-activation and the activation
    (gemm_gelu_aux) instead of the GEMM (whichever engine use_native picks) +
    the bias_gelu_fwd pass; timed once per shape under 'auto'."""
    if (_POLICY == "never" or not _GELU_AUX or M % 256 or N % 256 or K % 128
            or torch.device(dev).type != "cuda"):
        return False
    if _POLICY == "always":
        return True
    key = ("gelu_aux", M, N, K)
    hit = _choice.get(key)
    if hit is None and _fixed(key) is not None:
        hit = _choice[key] = _fixed(key)
    if hit is None:
        if torch.cuda.is_current_stream_capturing():
            return False
        C = _C()
        bf = torch.bfloat16
        a, b = torch.randn(M, K, device=dev, dtype=bf), torch.randn(N, K, device=dev, dtype=bf)
        u, h = torch.empty(M, N, device=dev, dtype=bf), torch.empty(M, N, device=dev, dtype=bf)
        bias = torch.randn(N, device=dev)
        if not C.gemm_gelu_aux(a, False, b, True, h, u, bias):
            _choice[key] = False
            return False
        native = use_native("fwd", M, N, K, dev)

        def theirs():
            if native:
                linear_fwd(a, b, out=u)
            else:
                torch.mm(a, b.t(), out=u)
            C.bias_gelu_fwd(u, bias, h)
        t_ours = _time(lambda: C.gemm_gelu_aux(a, False, b, True, h, u, bias))
        t_theirs = _time(theirs)
        hit = _choice[key] = t_ours <= t_theirs * (1.0 + _MARGIN)
        _timings[key] = (round(t_ours, 4), round(t_theirs, 4))
    return hit


def choices() -> dict:
    """{(role, M, N, K): (native chosen, (native ms, torch ms))}"""
    return {k: (v, _timings.get(k)) for k, v in _choice.items()}


def linear_fwd(x2, w16, bias=None, act: int = 0, out=None):
    out = torch.empty(x2.shape[0], w16.shape[0], device=x2.device, dtype=x2.dtype) if out is None else out
    if not _C().gemm_big(x2, False, w16, True, out, bias=bias, act=act):
        if bias is not None or act:
            raise ValueError("linear_fwd: epilogue needs the native kernel's shape contract")
        torch.mm(x2, w16.t(), out=out)
    return out


def linear_dx(gy2, w16, extra=None):
    """dx = gy2 @ w16 (+ extra, in place into `extra` when given)."""
    if extra is not None:
        if not _C().gemm_big(gy2, False, w16, False, extra, beta=1.0):
            extra.addmm_(gy2, w16)
        return extra
    out = torch.empty(gy2.shape[0], w16.shape[1], device=gy2.device, dtype=gy2.dtype)
    if not _C().gemm_big(gy2, False, w16, False, out):
        torch.mm(gy2, w16, out=out)
    return out


def linear_dw(gy2, x2, into=None):
    """dW[out, in] = gy2^T x2 in fp32 (accumulated into `into` when given)."""
    if into is None:
        into = torch.empty(gy2.shape[1], x2.shape[1], device=gy2.device, dtype=torch.float32)
        beta = 0.0
    else:
        beta = 1.0
    if not _C().gemm_big(gy2, True, x2, False, into, beta=beta, split_k=0):
        if beta:
            torch.addmm(into, gy2.t(), x2, out_dtype=torch.float32, out=into)
        else:
            torch.mm(gy2.t(), x2, out_dtype=torch.float32, out=into)
    return into
