"""Conv2d on the optimizer-maintained bf16 weight shadow, with a sunk wgrad.

The convolutions themselves stay on MIOpen (its implicit-GEMM MFMA solvers,
picked by solver search when `torch.backends.cudnn.benchmark` is on); what
this removes is the glue around them in a bf16-compute / fp32-master step:

* forward reads `weight._shadow` (bf16, same channels_last layout), which the
  fused optimizer rewrites in the same pass that updates the fp32 master --
  no per-step fp32->bf16 weight cast;
* backward asks MIOpen for (dx, dW) in one `convolution_backward` call and,
  when the weight is managed by DDP (ops.grad_sink), folds the bf16 dW into
  the fp32 bucket view with one mixed-dtype add -- no bf16->fp32 cast pass and
  no separate AccumulateGrad add;
* a 1x1 / stride-1 convolution on NHWC activations is a plain GEMM over the
  rows: y[NHW, cout] = x[NHW, cin] W^T, dx = dy W, dW = dy^T x.  Each of the
  three products picks, per shape and once (timed on the layer's own
  operands), between MIOpen and the GEMM engines: hipBLASLt (`torch.mm`) or
  the in-tree `gemm_big.hip` for y / dx, and for dW the in-tree GEMM with
  split-K accumulated straight into the fp32 bucket (MIOpen's atomic wrw
  solver adds zero-fill, scale and fp32 -> bf16 cast passes, then our bf16 ->
  fp32 add).  MIOpen keeps the early layers' forwards; the GEMMs win most
  input gradients (ResNet-50 B=128: 20-60 % per layer,
  profiles/resnet50_r4.md).  `DTF_CONV_GEMM`: auto (default) / never.
* a 3x3 / pad-1 / stride-1-or-2 convolution with 64-multiple channel counts
  may run on the in-tree implicit-GEMM kernel (`csrc/kernels/conv_igemm.hip`,
  MFMA, no im2col buffer): its forward, and for stride 1 its input gradient
  (the same convolution of dy with the flipped, channel-transposed filter),
  each chosen per shape against MIOpen by the same one-time timing.  The
  kernel can also emit the BatchNorm statistics partials of its output
  (`conv3x3(..., stats=)`).  `DTF_CONV_IGEMM`: auto (default) / never / always.
* BatchNorm statistics hand-off (`DTF_CONV_BN_STATS`, default on): the 3x3
  kernel and the 1x1 gemm_big forward (`dtfk_gemm_bn_stats`) write the
  per-channel sum / sum-of-squares partials of their output in the epilogue;
  the FusedBatchNorm2d consuming that output finalizes them instead of
  re-reading it.  Engine timing charges the engines without the epilogue
  (MIOpen, hipBLASLt) with that statistics pass.
Any other case (CPU, no shadow, eval under a different dtype) is plain
`nn.Conv2d`.
"""
from __future__ import annotations

import os
import weakref

import torch
import torch.nn.functional as F

from . import grad_sink

_POLICY = os.environ.get("DTF_CONV_GEMM", "auto")
_IGEMM = os.environ.get("DTF_CONV_IGEMM", "auto")
# a 3x3 forward on the in-tree kernel also writes its output's BatchNorm statistics
# partials; the FusedBatchNorm2d reading that output then skips its statistics pass
_BN_STATS = os.environ.get("DTF_CONV_BN_STATS", "1") != "0"
# strided 1x1 projections: forward / weight gradient on the implicit GEMM's
# strided loads, chosen per shape against MIOpen (0, default: no gathered copy;
# ResNet-50 9,391-9,413 vs 9,258-9,302 img/s same box, scripts/sessions/gpu_r6q.sh),
# or gather the strided pixels once and run them as GEMMs over the copy (1)
_S2_GATHER = os.environ.get("DTF_CONV_S2_GATHER", "0") != "0"
_handoff = {}   # id(conv output) -> (partials, P): from _ShadowConv.forward to ShadowConv2d.forward
_choice: dict = {}
_timings: dict = {}


def _gemm_ok(x, w16, stride, padding, dilation, groups) -> bool:
    """A 1x1 / stride-1 / unpadded / ungrouped conv on channels_last bf16 rows."""
    return (w16.shape[2] == 1 and w16.shape[3] == 1 and tuple(stride) == (1, 1) and tuple(padding) == (0, 0)
            and groups == 1 and x.is_cuda and x.dtype == torch.bfloat16
            and x.is_contiguous(memory_format=torch.channels_last)
            and (x.shape[0] * x.shape[2] * x.shape[3]) % 64 == 0)


def _rows(t):
    """[N, C, H, W] channels_last -> its [N*H*W, C] row view (no copy)."""
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])


def _cl_empty(n, c, h, w, like):
    return torch.empty((n, c, h, w), device=like.device, dtype=like.dtype, memory_format=torch.channels_last)


def _fwd_gemm(engine, x, w16):
    y = _cl_empty(x.shape[0], w16.shape[0], x.shape[2], x.shape[3], x)
    x2, w2, y2 = _rows(x), w16.view(w16.shape[0], w16.shape[1]), _rows(y)
    if engine != "gemm_big" or not _C().gemm_big(x2, False, w2, True, y2):
        torch.mm(x2, w2.t(), out=y2)
    return y


def _fwd_gemm_stats(x, w16):
    """1x1 forward on gemm_big with the BatchNorm statistics partials of y in
    the epilogue: (y, part [2, P, cout], P), or None outside the kernel's contract."""
    y = _cl_empty(x.shape[0], w16.shape[0], x.shape[2], x.shape[3], x)
    x2, w2, y2 = _rows(x), w16.view(w16.shape[0], w16.shape[1]), _rows(y)
    P = int(_C().gemm_bn_stat_rows(x2.shape[0]))
    part = torch.empty((2, P, w16.shape[0]), device=x.device, dtype=torch.float32)
    if not _C().gemm_bn_stats(x2, False, w2, True, y2, part):
        return None
    return y, part, P


def _stat_pass(y):
    """The statistics pass a BatchNorm runs over a conv output that came without
    partials (what the engine timing charges the engines without an epilogue)."""
    C = _C()
    part = torch.empty(2 * C.bn_partial_rows(y.numel() // y.shape[1], y.shape[1]) * y.shape[1],
                       device=y.device, dtype=torch.float32)
    C.bn_stat_partials(y, part)


def _dx_gemm(engine, dy, w16, x_shape, into=None):
    """dx = dy W; with `into` (a channels_last bf16 gradient of x from another
    branch) accumulated in place: dx = into + dy W, one GEMM with beta = 1."""
    acc = into is not None and into.dtype == dy.dtype and into.is_contiguous(memory_format=torch.channels_last)
    if engine == "igemm":     # the in-tree implicit GEMM (1x1: dy times the transposed filter), accumulating
        return conv3x3_dx(dy, w16, x_shape, into=into if acc else None) if acc or into is None else \
            conv3x3_dx(dy, w16, x_shape) + into
    dx = into if acc else _cl_empty(x_shape[0], x_shape[1], x_shape[2], x_shape[3], dy)
    dy2, w2, dx2 = _rows(dy), w16.view(w16.shape[0], w16.shape[1]), _rows(dx)
    if engine != "gemm_big" or not _C().gemm_big(dy2, False, w2, False, dx2, beta=1.0 if acc else 0.0):
        if acc:
            dx2.addmm_(dy2, w2)
        else:
            torch.mm(dy2, w2, out=dx2)
    if into is not None and not acc:
        dx = dx + into
    return dx


def _C():
    from .. import _native
    return _native.load()


def igemm_ok(x, w16, stride, padding, dilation, groups) -> bool:
    """A 3x3 / pad 1 / stride 1 or 2 conv the in-tree implicit GEMM takes -- or,
    without the strided-pixel gather (DTF_CONV_S2_GATHER=0), a 1x1 / pad 0 /
    stride 2 projection (its strided loads gather the pixels in place)."""
    if w16.dim() != 4 or w16.shape[2] != w16.shape[3]:
        return False
    k = w16.shape[2]
    shape_ok = ((k == 3 and tuple(padding) == (1, 1) and stride[0] in (1, 2))
                or (k == 1 and not _S2_GATHER and tuple(padding) == (0, 0) and stride[0] == 2))
    return (_IGEMM != "never" and shape_ok
            and tuple(dilation) == (1, 1) and groups == 1
            and stride[0] == stride[1] and x.is_cuda and x.dtype == torch.bfloat16
            and w16.dtype == torch.bfloat16 and x.is_contiguous(memory_format=torch.channels_last)
            and w16.is_contiguous(memory_format=torch.channels_last)
            and bool(_C().conv3x3_supported(x, w16, int(stride[0]))))


def igemm1_ok(x, w16) -> bool:
    """A 1x1 / stride-1 conv (the GEMM path's shapes) the in-tree implicit GEMM takes."""
    return (_IGEMM != "never" and w16.dim() == 4 and w16.shape[2] == 1 and w16.shape[3] == 1
            and w16.is_contiguous(memory_format=torch.channels_last) and bool(_C().conv3x3_supported(x, w16, 1)))


def conv3x3(x, w16, stride: int = 1, stats=None, out=None, bn: int = 0, accumulate: bool = False,
            bn_x=None, bn_stats=None, bn_res=None):
    """y = conv2d(x, w16, stride, padding=k//2) on the in-tree implicit GEMM
    (channels_last bf16; w16 3x3 or 1x1).  `stats`: an fp32 [2, P, Cout]
    buffer (P = `conv3x3_stat_rows`) that receives per-channel sums of y and
    y^2 per 128-row tile -- the partials csrc/kernels/bn.hip's finalize
    reduces.  `bn`: output-channel tile width (64 / 128; 0 = the kernel's
    choice).  `accumulate`: out += the convolution.  `bn_x` / `bn_stats`: y is
    the output gradient of a BatchNorm + ReLU whose input was bn_x (stats
    [4, Cout]); y is stored ReLU-masked and `stats` receives that BN
    backward's partials (sum g, sum g * x_hat) instead.  `bn_res` (with
    accumulate): that BN added this residual before the ReLU, and `out` holds
    the residual branch's gradient the convolution is added onto first."""
    N, _, H, W = x.shape
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    y = _cl_empty(N, w16.shape[0], Ho, Wo, x) if out is None else out
    _C().conv3x3_fwd(x, w16, y, stats, stride, bn, accumulate, bn_x, bn_stats, bn_res)
    return y


def conv3x3_stat_rows(x, stride: int = 1) -> int:
    return int(_C().conv3x3_tiles(x.shape[0], x.shape[2], x.shape[3], stride))


# flipped filters of the input gradients: id(w16) -> [weakref(w16), wt, w16._version at the flip].
# The fused optimizer rewrites a shadow in place and bumps its version
# (optim.FusedOptimizer.step), so after a step the first input gradient
# re-flips every registered filter in ONE launch (conv_wflip_multi) instead
# of one wflip launch per conv backward (~5 us each, 40 per ResNet-50 step).
_FLIP_CACHE = os.environ.get("DTF_CONV_FLIP_CACHE", "1") != "0"
_flips: dict = {}
_flip_tab: dict = {"key": None}


def _flipped(w16):
    ks = w16.shape[2]
    if not _FLIP_CACHE:
        wt = torch.empty((w16.shape[1], w16.shape[0], ks, ks), device=w16.device, dtype=w16.dtype,
                         memory_format=torch.channels_last)
        _C().conv3x3_wflip(w16, wt)
        return wt
    ent = _flips.get(id(w16))
    if ent is None or ent[0]() is not w16:
        wt = torch.empty((w16.shape[1], w16.shape[0], ks, ks), device=w16.device, dtype=w16.dtype,
                         memory_format=torch.channels_last)
        ent = _flips[id(w16)] = [weakref.ref(w16), wt, None]
    if ent[2] == w16._version:
        return ent[1]
    stale = []
    for k, e in list(_flips.items()):
        w = e[0]()
        if w is None:
            del _flips[k]
        elif e[2] != w._version and w.device == w16.device:
            stale.append((w, e))
    key = tuple((w.data_ptr(), e[1].data_ptr()) for w, e in stale)
    if _flip_tab["key"] != key and torch.cuda.is_current_stream_capturing():
        # no host-built table inside a capture: this filter alone
        _C().conv3x3_wflip(w16, ent[1])
        ent[2] = w16._version
        return ent[1]
    if _flip_tab["key"] != key:
        rows, tiles = [], []
        for i, (w, e) in enumerate(stale):
            K_, C_, ks_ = w.shape[0], w.shape[1], w.shape[2]
            rows.append([w.data_ptr(), e[1].data_ptr(), K_, C_, ks_])
            tiles.extend([i, rs, k0, c0] for rs in range(ks_ * ks_) for k0 in range(0, K_, 64)
                         for c0 in range(0, C_, 64))
        _flip_tab.update(key=key, tab=torch.tensor(rows, dtype=torch.int64).to(w16.device),
                         tiles=torch.tensor(tiles, dtype=torch.int32).reshape(-1, 4).to(w16.device),
                         refs=[e[1] for _, e in stale])
    _C().conv_wflip_multi(_flip_tab["tab"], _flip_tab["tiles"])
    for w, e in stale:
        e[2] = w._version
    return ent[1]


def _bnb_fits(bnb, into, x_shape) -> bool:
    """The BN-backward epilogue applies: the BN's tensors have x's shape, and a
    residual BN comes with the residual branch's gradient to add onto (a plain
    one without)."""
    if bnb is None or tuple(bnb.x.shape) != tuple(x_shape) or bnb.stats.numel() != 4 * x_shape[1]:
        return False
    if bnb.res is None:
        return into is None
    return (into is not None and tuple(bnb.res.shape) == tuple(x_shape) and tuple(into.shape) == tuple(x_shape)
            and into.dtype == torch.bfloat16 and into.is_contiguous(memory_format=torch.channels_last)
            and bnb.res.is_contiguous(memory_format=torch.channels_last))


def conv3x3_dx(dy, w16, x_shape, into=None, bnb=None):
    """Input gradient of a stride-1 3x3 (or 1x1) conv: the same convolution of
    dy with the flipped, channel-transposed filter; `into` (a channels_last bf16
    gradient of x from another branch) is accumulated in the epilogue.  `bnb`
    (ops.bn.BwdSlot of the BatchNorm (+ residual) + ReLU that produced x): dx
    is returned ReLU-masked and the epilogue writes that BN backward's partials
    into the slot, so the BN's backward skips its own pass over the gradient
    (with a residual BN, `into` must be the residual branch's gradient)."""
    wt = _flipped(w16)
    if _bnb_fits(bnb, into, x_shape):
        P = conv3x3_stat_rows(dy, 1)
        part = torch.empty((2, P, x_shape[1]), device=dy.device, dtype=torch.float32)
        dx = into if into is not None else _cl_empty(x_shape[0], x_shape[1], x_shape[2], x_shape[3], dy)
        conv3x3(dy, wt, 1, stats=part, out=dx, accumulate=into is not None, bn_x=bnb.x, bn_stats=bnb.stats,
                bn_res=bnb.res)
        bnb.part, bnb.g, bnb.g_version = (part, P), dx, dx._version
        return dx
    if into is not None:
        return conv3x3(dy, wt, 1, out=into, accumulate=True)
    dx = _cl_empty(x_shape[0], x_shape[1], x_shape[2], x_shape[3], dy)
    return conv3x3(dy, wt, 1, out=dx)


def _fuse_bnb(bnb, dx_eng, key, x) -> bool:
    """Route a 1x1 input gradient onto the implicit GEMM for the BN-backward
    epilogue: when it is the chosen engine, or when its measured deficit is
    below the HBM passes the epilogue saves (one over x for a plain BN, two
    with a residual: the partials pass re-reads dy, x (and res) and writes g)."""
    if dx_eng == "igemm":
        return True
    t = _timings.get(("dx",) + key)
    if not t or "igemm" not in t:
        return False
    passes = 2 if bnb.res is not None else 1
    return t["igemm"] - min(t.values()) <= passes * x.numel() * 2 / 5e9   # ms at ~5 TB/s


def conv3x3_dw(dy, x, stride: int, into=None, ks=None):
    """fp32 weight gradient of y = conv3x3(x, w, stride) for y's gradient dy,
    accumulated into `into` (an fp32 [Cout, Cin, 3, 3] tensor, contiguous or
    channels_last) or into a fresh zeroed one."""
    if into is None:
        ks = 3 if ks is None else ks
        into = torch.zeros((dy.shape[1], x.shape[1], ks, ks), device=dy.device, dtype=torch.float32)
    _C().conv3x3_wgrad(dy, x, into, stride)
    return into


def _dw3_engine(dy, x, w16, stride: int) -> str:
    if _IGEMM == "always":
        return "igemm"
    key = (tuple(x.shape), w16.shape[0], stride, w16.shape[2])
    if ("dw3",) + key not in _choice:
        if _POLICY == "never":
            return "miopen"
        # the accumulator in the layout of the .grad it stands for (the weight's)
        fmt = torch.channels_last if w16.is_contiguous(memory_format=torch.channels_last) else torch.contiguous_format
        k, pad = w16.shape[2], w16.shape[2] // 2
        acc = torch.zeros((w16.shape[0], w16.shape[1], k, k), device=x.device, dtype=torch.float32).contiguous(
            memory_format=fmt)

        def miopen():
            dw = torch.ops.aten.convolution_backward(dy, x, w16, None, (stride, stride), (pad, pad), (1, 1), False,
                                                     [0, 0], 1, [False, True, False])[1]
            acc.add_(dw.float())
        return _pick("dw3", key, {"miopen": miopen, "igemm": lambda: conv3x3_dw(dy, x, stride, into=acc)})
    return _choice[("dw3",) + key]


def _fwd3_engine(x, w16, stride: int) -> str:
    if _IGEMM == "always":
        return "igemm"
    key = (tuple(x.shape), w16.shape[0], stride, w16.shape[2])
    pad = w16.shape[2] // 2
    if ("fwd3",) + key not in _choice:
        if _POLICY == "never":
            return "miopen"
        if _BN_STATS:   # the igemm epilogue writes the BatchNorm partials MIOpen's output needs a pass for
            P = conv3x3_stat_rows(x, stride)
            part = torch.empty((2, P, w16.shape[0]), device=x.device, dtype=torch.float32)
            return _pick("fwd3", key, {"miopen": lambda: _stat_pass(F.conv2d(x, w16, None, stride, pad)),
                                       "igemm": lambda: conv3x3(x, w16, stride, stats=part)})
        return _pick("fwd3", key, {"miopen": lambda: F.conv2d(x, w16, None, stride, pad),
                                   "igemm": lambda: conv3x3(x, w16, stride)})
    return _choice[("fwd3",) + key]


def _dx3_engine(dy, x, w16) -> str:
    if _IGEMM == "always":
        return "igemm"
    key = (tuple(x.shape), w16.shape[0], 1)
    if ("dx3",) + key not in _choice:
        if _POLICY == "never":
            return "miopen"
        return _pick("dx3", key, {"miopen": lambda: torch.ops.aten.convolution_backward(
                         dy, x, w16, None, (1, 1), (1, 1), (1, 1), False, [0, 0], 1, [True, False, False]),
                     "igemm": lambda: conv3x3_dx(dy, w16, x.shape)})
    return _choice[("dx3",) + key]


def _pick(role, key, cands) -> str:
    """Fastest of `cands` {name: fn} for (role, key), timed once (MIOpen first)."""
    k = (role,) + key
    hit = _choice.get(k)
    if hit is None:
        if _POLICY == "never" or torch.cuda.is_current_stream_capturing():
            return "miopen"
        from . import big_gemm
        t = {name: big_gemm._time(fn, reps=3) for name, fn in cands.items()}
        hit = _choice[k] = min(t, key=t.get)
        _timings[k] = {n: round(v, 4) for n, v in t.items()}
    return hit


def _fwd_engine(x, w16) -> str:
    if _POLICY == "never":
        return "miopen"
    key = (tuple(x.shape), w16.shape[0])
    if ("fwd",) + key not in _choice:
        if _BN_STATS and _fwd_gemm_stats(x, w16) is not None:
            # gemm_big / the implicit GEMM hand their output's BatchNorm partials over;
            # the others leave a statistics pass
            cands = {"miopen": lambda: _stat_pass(F.conv2d(x, w16)),
                     "hipblaslt": lambda: _stat_pass(_fwd_gemm("hipblaslt", x, w16)),
                     "gemm_big": lambda: _fwd_gemm_stats(x, w16)}
            if igemm1_ok(x, w16):
                part = torch.empty((2, conv3x3_stat_rows(x, 1), w16.shape[0]), device=x.device, dtype=torch.float32)
                cands["igemm"] = lambda: conv3x3(x, w16, 1, stats=part)
        else:
            cands = {"miopen": lambda: F.conv2d(x, w16),
                     "hipblaslt": lambda: _fwd_gemm("hipblaslt", x, w16),
                     "gemm_big": lambda: _fwd_gemm("gemm_big", x, w16)}
            if igemm1_ok(x, w16):
                cands["igemm"] = lambda: conv3x3(x, w16, 1)
        return _pick("fwd", key, cands)
    return _choice[("fwd",) + key]


def _dx_engine(dy, x, w16) -> str:
    if _POLICY == "never":
        return "miopen"
    key = (tuple(x.shape), w16.shape[0])
    if ("dx",) + key not in _choice:
        cands = {"miopen": lambda: torch.ops.aten.convolution_backward(
                     dy, x, w16, None, (1, 1), (0, 0), (1, 1), False, [0, 0], 1, [True, False, False]),
                 "hipblaslt": lambda: _dx_gemm("hipblaslt", dy, w16, x.shape),
                 "gemm_big": lambda: _dx_gemm("gemm_big", dy, w16, x.shape)}
        if igemm1_ok(x, w16) and dy.is_contiguous(memory_format=torch.channels_last):
            cands["igemm"] = lambda: _dx_gemm("igemm", dy, w16, x.shape)
        return _pick("dx", key, cands)
    return _choice[("dx",) + key]


def _dw_engine(dy, x, w16) -> str:
    """The in-tree GEMM accumulating into an fp32 target vs MIOpen's weight
    gradient + the bf16 -> fp32 add."""
    if _POLICY == "never":
        return "miopen"
    key = (tuple(x.shape), w16.shape[0])
    if ("dw",) + key not in _choice:
        from . import big_gemm
        acc = torch.zeros(w16.shape[0], w16.shape[1], device=x.device, dtype=torch.float32)
        x2, dy2 = _rows(x), _rows(dy)

        def miopen():
            dw = torch.ops.aten.convolution_backward(dy, x, w16, None, (1, 1), (0, 0), (1, 1), False, [0, 0], 1,
                                                     [False, True, False])[1]
            acc.add_(dw.view(acc.shape).float())
        cands = {"miopen": miopen, "gemm_big": lambda: big_gemm.linear_dw(dy2, x2, into=acc)}
        if igemm1_ok(x, w16):
            acc4 = acc.view(w16.shape[0], w16.shape[1], 1, 1)
            cands["igemm"] = lambda: conv3x3_dw(dy, x, 1, into=acc4)
        return _pick("dw", key, cands)
    return _choice[("dw",) + key]


def choices() -> dict:
    """{(role, x shape, cout): (engine, {engine: ms})}"""
    return {k: (v, _timings.get(k)) for k, v in _choice.items()}


class XGradShare:
    """Two 1x1 convolutions reading the same input (a downsampling bottleneck's
    conv1 and projection): whichever backward runs first deposits its input
    gradient, the second folds its own in and returns the sum -- a GEMM with
    beta = 1, or, for the stride-2 projection, its compact gradient added onto
    the strided pixels (strided_add), instead of a zero-filled full-size dx from
    MIOpen plus an autograd add."""
    __slots__ = ("part",)

    def __init__(self):
        self.part = None   # ("full", dx) or ("strided", compact dx, stride)

    def take(self):
        p, self.part = self.part, None
        return p


def _strided_ok(x, w16, stride, padding, dilation, groups) -> bool:
    """A 1x1 / stride-s / unpadded conv whose input gradient is a GEMM over the
    strided pixels."""
    return (w16.shape[2] == 1 and w16.shape[3] == 1 and tuple(padding) == (0, 0) and groups == 1
            and stride[0] == stride[1] and stride[0] > 1 and x.is_cuda and x.dtype == torch.bfloat16
            and x.is_contiguous(memory_format=torch.channels_last) and x.shape[1] % 8 == 0)


def _s2_ok(x, w16, stride, padding, dilation, groups) -> bool:
    """A strided 1x1 conv (unpadded, ungrouped) whose forward / weight gradient
    may run as GEMMs over the gathered strided pixels (DTF_CONV_GEMM=never: off)."""
    return (_S2_GATHER and _POLICY != "never" and _strided_ok(x, w16, stride, padding, dilation, groups)
            and tuple(dilation) == (1, 1))


def _fwd_igemm1(x, w16):
    """1x1 forward on the implicit GEMM, with the BatchNorm partials hand-off."""
    if _BN_STATS:
        P = conv3x3_stat_rows(x, 1)
        part = torch.empty((2, P, w16.shape[0]), device=x.device, dtype=torch.float32)
        y = conv3x3(x, w16, 1, stats=part)
        _handoff[id(y)] = (part, P)
        return y
    return conv3x3(x, w16, 1)


class _ShadowConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, w16, stride, padding, dilation, groups, slot=None, share=None, bnb=None):
        ctx.save_for_backward(x, w16)
        ctx.conf = (stride, padding, dilation, groups)
        ctx.w = w
        ctx.slot = slot
        ctx.share = share
        ctx.bnb = bnb     # ops.bn.BwdSlot of the BatchNorm + ReLU that produced x
        ctx.gemm = _gemm_ok(x, w16, stride, padding, dilation, groups)
        ctx.xs = None
        if not ctx.gemm and _s2_ok(x, w16, stride, padding, dilation, groups):
            # strided 1x1 (ResNet's downsampling projection): gather the strided
            # pixels once; forward and weight gradient are then plain GEMMs over
            # them (the input gradient keeps the strided-GEMM / MIOpen path)
            xs = x[:, :, ::stride[0], ::stride[1]].contiguous(memory_format=torch.channels_last)
            if _gemm_ok(xs, w16, (1, 1), (0, 0), dilation, groups):
                ctx.xs = xs
                eng = _fwd_engine(xs, w16)
                if eng == "igemm":
                    return _fwd_igemm1(xs, w16)
                if eng == "gemm_big" and _BN_STATS:
                    r = _fwd_gemm_stats(xs, w16)
                    if r is not None:
                        _handoff[id(r[0])] = (r[1], r[2])
                        return r[0]
                if eng != "miopen":
                    return _fwd_gemm(eng, xs, w16)
                return F.conv2d(xs, w16)
        if ctx.gemm:
            eng = _fwd_engine(x, w16)
            if eng == "igemm":
                return _fwd_igemm1(x, w16)
            if eng == "gemm_big" and _BN_STATS:
                r = _fwd_gemm_stats(x, w16)
                if r is not None:
                    _handoff[id(r[0])] = (r[1], r[2])
                    return r[0]
            if eng != "miopen":
                return _fwd_gemm(eng, x, w16)
        ctx.igemm = igemm_ok(x, w16, stride, padding, dilation, groups)
        if ctx.igemm and _fwd3_engine(x, w16, int(stride[0])) == "igemm":
            if _BN_STATS:
                s = int(stride[0])
                P = conv3x3_stat_rows(x, s)
                part = torch.empty((2, P, w16.shape[0]), device=x.device, dtype=torch.float32)
                y = conv3x3(x, w16, s, stats=part)
                _handoff[id(y)] = (part, P)
                return y
            return conv3x3(x, w16, int(stride[0]))
        return F.conv2d(x, w16, None, stride, padding, dilation, groups)

    @staticmethod
    def backward(ctx, dy):
        x, w16 = ctx.saved_tensors
        stride, padding, dilation, groups = ctx.conf
        need_x = ctx.needs_input_grad[0]
        need_w = ctx.needs_input_grad[1]
        dy = dy.to(w16.dtype)
        w = ctx.w
        gemm = ctx.gemm and dy.is_contiguous(memory_format=torch.channels_last)
        share = ctx.share if need_x else None
        other = share.take() if share is not None else None    # what the pair's first backward deposited
        first = share is not None and other is None
        strided = (share is not None and dy.is_contiguous(memory_format=torch.channels_last)
                   and _strided_ok(x, w16, stride, padding, dilation, groups))
        xs = getattr(ctx, "xs", None)     # the strided 1x1's gathered pixels (its weight gradient is a GEMM over them)
        xw = xs if xs is not None else x
        gw = (ctx.gemm or xs is not None) and dy.is_contiguous(memory_format=torch.channels_last)
        dx_eng = _dx_engine(dy, x, w16) if gemm and need_x else "miopen"
        dw_eng = _dw_engine(dy, xw, w16) if gw and need_w else "miopen"
        dx3 = (_dx3_engine(dy, x, w16) if need_x and getattr(ctx, "igemm", False) and tuple(stride) == (1, 1)
               and dy.is_contiguous(memory_format=torch.channels_last) else "miopen")
        dw3 = (_dw3_engine(dy, x, w16, int(stride[0])) if need_w and getattr(ctx, "igemm", False)
               and dy.is_contiguous(memory_format=torch.channels_last) else "miopen")
        extra = ctx.slot.take() if ctx.slot is not None else None   # a residual branch's gradient of x
        if other is not None and other[0] == "full":    # the pair's full-size gradient of x
            extra = other[1] if extra is None else extra.add_(other[1])
        # the BatchNorm (+ residual) + ReLU that produced x takes its backward
        # partials from this input gradient's epilogue (not for a shared x: the
        # pair's other gradient would be missing from the mask's input)
        bnb = ctx.bnb if share is None else None
        bnb_ok = need_x and bnb is not None and not strided and _bnb_fits(bnb, extra, x.shape)
        fuse1 = (bnb_ok and dx3 != "igemm" and gemm and igemm1_ok(x, w16)
                 and _fuse_bnb(bnb, dx_eng, (tuple(x.shape), w16.shape[0]), x))
        # MIOpen's share: one convolution_backward call for whatever stays on it
        mx = need_x and dx_eng == "miopen" and not strided and dx3 == "miopen" and not fuse1
        mw = need_w and dw_eng == "miopen" and dw3 == "miopen"
        dx = dw = None
        if mx or mw:
            dx, dw, _ = torch.ops.aten.convolution_backward(dy, x, w16, None, stride, padding, dilation, False,
                                                            [0, 0], groups, [mx, mw, False])
        if strided:
            # the input gradient lives on the strided pixels only: [N*Ho*Wo, Cin] = dy W
            comp = _cl_empty(x.shape[0], x.shape[1], dy.shape[2], dy.shape[3], dy)
            torch.mm(_rows(dy), w16.view(w16.shape[0], w16.shape[1]), out=_rows(comp))
            if extra is None:            # first of the pair: the other conv adds its gradient onto this later
                share.part = ("strided", comp, stride[0])
            else:
                _C().strided_add(extra, comp, stride[0])
                dx = extra
        elif need_x and dx3 == "igemm" and bnb_ok:
            dx = conv3x3_dx(dy, w16, x.shape, into=extra, bnb=bnb)
        elif need_x and dx3 == "igemm":
            dx = conv3x3_dx(dy, w16, x.shape)
            if extra is not None:
                dx = dx.add_(extra)
        elif fuse1:
            dx = conv3x3_dx(dy, w16, x.shape, into=extra, bnb=bnb)
        elif need_x and not mx:
            dx = _dx_gemm(dx_eng, dy, w16, x.shape, into=extra)
        elif need_x and extra is not None:
            dx = dx + extra
        if other is not None and other[0] == "strided":
            _C().strided_add(dx, other[1], other[2])
        if first and not strided:        # first of the pair: hand the full gradient to the second
            share.part, dx = ("full", dx), None
        if not need_w:
            return dx, None, None, None, None, None, None, None, None, None
        # every weight-gradient path below accumulates into a contiguous or a
        # channels_last fp32 .grad (the DDP bucket view mirrors the weight's layout:
        # channels_last 3x3 filters included)
        sink = grad_sink.enabled(w) and (w.grad is None or w.grad.is_contiguous()
                                         or w.grad.is_contiguous(memory_format=torch.channels_last))
        if dw3 == "igemm":      # the in-tree weight gradient accumulates straight into fp32
            if sink:
                conv3x3_dw(dy, x, int(stride[0]), into=grad_sink.target(w))
                grad_sink.done(w)
                return dx, None, None, None, None, None, None, None, None, None
            return (dx, conv3x3_dw(dy, x, int(stride[0]), ks=w16.shape[2]).to(w.dtype), None, None, None, None, None,
                    None, None, None)
        if not mw and dw_eng == "igemm":     # the 1x1 implicit GEMM's weight gradient, straight into fp32
            if sink:
                conv3x3_dw(dy, xw, 1, into=grad_sink.target(w))
                grad_sink.done(w)
                return dx, None, None, None, None, None, None, None, None, None
            return dx, conv3x3_dw(dy, xw, 1, ks=1).to(w.dtype), None, None, None, None, None, None, None, None
        if not mw:
            from . import big_gemm
            if sink:
                g = grad_sink.target(w)
                big_gemm.linear_dw(_rows(dy), _rows(xw), into=g.view(g.shape[0], g.shape[1]))
                grad_sink.done(w)
                return dx, None, None, None, None, None, None, None, None, None
            return (dx, big_gemm.linear_dw(_rows(dy), _rows(xw)).view(w.shape).to(w.dtype), None, None, None, None,
                    None, None, None, None)
        if sink:
            # bf16 -> fp32 first: a mixed-dtype add_ into the fp32 .grad runs PyTorch's
            # vectorized_templated kernel at ~45 us for a 9-37K element filter on this
            # stack (3.9 us as a copy + same-dtype add; profiles/resnet50_sink_add_r5.txt)
            grad_sink.target(w).add_(dw.float())
            grad_sink.done(w)
            return dx, None, None, None, None, None, None, None, None, None
        return dx, dw.to(w.dtype), None, None, None, None, None, None, None, None


class ShadowConv2d(torch.nn.Conv2d):
    """nn.Conv2d that computes with `weight._shadow` when one is attached."""

    def forward(self, x, grad_slot=None, share=None):
        """`grad_slot` (ops.transformer.GradSlot): another branch's gradient of x,
        deposited by its producer during backward, is accumulated into this
        conv's input gradient (the residual add of a bottleneck's identity path).
        `share` (XGradShare): this conv and one other read the same x and fold
        their input gradients into one tensor.  Both only take effect on the
        shadow path, which the caller must ensure (`on_shadow_path`)."""
        if self.on_shadow_path(x):
            y = _ShadowConv.apply(x, self.weight, self.weight._shadow, self.stride, self.padding, self.dilation,
                                  self.groups, grad_slot, share, getattr(x, "_dtf_bn_bwd", None))
            if _handoff:
                st = _handoff.pop(id(y), None)
                _handoff.clear()
                if st is not None:
                    # read by the FusedBatchNorm2d that consumes y, only while y is
                    # unmodified (an in-place op between the conv and the BN bumps
                    # _version and the BN recomputes its statistics)
                    y._dtf_bn_part = (st, y._version)
            return y
        w16 = getattr(self.weight, "_shadow", None)
        if (w16 is not None and x.is_cuda and self.bias is None and self.padding_mode == "zeros"
                and isinstance(self.padding, tuple)):
            return _ShadowConv.apply(x.to(w16.dtype), self.weight, w16, self.stride, self.padding, self.dilation,
                                     self.groups)
        return super().forward(x)

    def on_shadow_path(self, x) -> bool:
        """x goes straight into _ShadowConv (the path that honours grad_slot / share)."""
        w16 = getattr(self.weight, "_shadow", None)
        return (w16 is not None and x.is_cuda and x.dtype == w16.dtype and self.bias is None
                and self.padding_mode == "zeros" and isinstance(self.padding, tuple))


def attach_shadows(module: torch.nn.Module, optimizer=None, dtype=torch.bfloat16):
    """Give every ShadowConv2d weight a bf16 shadow kept current by `optimizer`
    (a fused optimizer's attach_shadow), or a one-off copy without one."""
    for m in module.modules():
        if isinstance(m, ShadowConv2d):
            w = m.weight
            if getattr(w, "_shadow", None) is None:
                w._shadow = torch.empty_like(w, dtype=dtype)
            if optimizer is not None:
                optimizer.attach_shadow(w, w._shadow)
            else:
                with torch.no_grad():
                    w._shadow.copy_(w)
