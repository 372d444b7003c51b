"""A small deferred-execution tensor layer with TF-1 graph semantics.

The reference builds TF graphs (placeholders, Variables under name scopes,
matmul/add/sigmoid/softmax, reduce_mean, ...) and evaluates them with
`sess.run(fetches, feed_dict)` (example.py:69-170; lr2.py:363-446).  This
module keeps that programming model -- so the reference scripts port almost
line by line -- while executing eagerly on PyTorch-ROCm tensors when a fetch
is run:

* `Tensor` nodes record (fn, inputs); `Session.run` evaluates the requested
  fetches once per call with memoisation (a run's loss and accuracy share the
  forward pass), autograd flows through Variables;
* `Variable`s own a device tensor (GPU when present), carry TF names
  (`weights/Variable_1:0`) and live in the GLOBAL/TRAINABLE/LOCAL collections,
  which the Saver uses for TF-format checkpoints;
* matmul dispatches to the framework's MFMA GEMM (`ops.linear_act`) on GPU.
"""
from __future__ import annotations

import contextlib
import threading
from collections import defaultdict
from typing import Any, Callable, Dict, List, Optional, Sequence

import numpy as np
import torch

# ----------------------------------------------------------------------- dtypes
float32 = torch.float32
float64 = torch.float64
float16 = torch.float16
bfloat16 = torch.bfloat16
int32 = torch.int32
int64 = torch.int64
uint8 = torch.uint8
bool_ = torch.bool
string = "string"

GLOBAL_VARIABLES = "variables"
TRAINABLE_VARIABLES = "trainable_variables"
LOCAL_VARIABLES = "local_variables"
SUMMARIES = "summaries"
QUEUE_RUNNERS = "queue_runners"
GLOBAL_STEP = "global_step"
UPDATE_OPS = "update_ops"


def default_device() -> torch.device:
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


class Graph:
    """Name scopes, collections, unique names and the device-placement stack."""

    def __init__(self):
        self._collections: Dict[str, List[Any]] = defaultdict(list)
        self._names: Dict[str, int] = {}
        self._scope: List[str] = []
        self._var_scope: List[str] = []
        self._var_reuse: List[bool] = []
        self._devices: List[Any] = []
        self._vars_by_name: Dict[str, "Variable"] = {}
        self.seed: Optional[int] = None
        self._op_seed = 0
        self.device = default_device()
        self.finalized = False
        self._nodes: List["Tensor"] = []          # creation order (GraphDef node order)

    @contextlib.contextmanager
    def as_default(self):
        prev = getattr(_local, "graph", None)
        _local.graph = self
        try:
            yield self
        finally:
            _local.graph = prev

    def unique_name(self, name: str) -> str:
        full = "/".join(self._scope + [name]) if self._scope else name
        n = self._names.get(full, 0)
        self._names[full] = n + 1
        return full if n == 0 else f"{full}_{n}"

    def add_to_collection(self, key, value):
        self._collections[key].append(value)

    def get_collection(self, key, scope: Optional[str] = None):
        vals = list(self._collections.get(key, []))
        if scope:
            vals = [v for v in vals if getattr(v, "name", "").startswith(scope)]
        return vals

    def get_collection_ref(self, key):
        return self._collections[key]

    def finalize(self):
        self.finalized = True

    def as_graph_def(self) -> bytes:
        """Serialized tensorflow.GraphDef of the nodes built so far
        (compat/meta_graph.py)."""
        from .meta_graph import graph_def_bytes

        return graph_def_bytes(self)

    def get_operations(self):
        return list(self._nodes)

    def get_tensor_by_name(self, name: str):
        idx = self.__dict__.get("_name_index")
        if idx is None or idx[0] != len(self._nodes):
            m = {}
            for t in self._nodes:
                m[t.name] = t
                m.setdefault(t.name[:-2], t)
            idx = self._name_index = (len(self._nodes), m)
        t = idx[1].get(name)
        if t is None:
            raise KeyError(f"The name '{name}' refers to a Tensor which does not exist")
        return t

    def next_seed(self):
        self._op_seed += 1
        if self.seed is None:
            return None
        return (self.seed * 1000003 + self._op_seed) % (2 ** 31)


_local = threading.local()


def get_default_graph() -> Graph:
    g = getattr(_local, "graph", None)
    if g is None:
        g = _local.graph = Graph()
    return g


def reset_default_graph():
    _local.graph = Graph()


def set_random_seed(seed: int):
    get_default_graph().seed = int(seed)


@contextlib.contextmanager
def name_scope(name: str):
    g = get_default_graph()
    scope = g.unique_name(name) if name else None
    if scope:
        g._scope.append(scope.split("/")[-1])
    try:
        yield scope
    finally:
        if scope:
            g._scope.pop()


@contextlib.contextmanager
def variable_scope(name: str, reuse: Optional[bool] = None):
    g = get_default_graph()
    g._var_scope.append(name)
    g._scope.append(name)
    g._var_reuse.append(bool(reuse))
    try:
        yield name
    finally:
        g._var_scope.pop()
        g._scope.pop()
        g._var_reuse.pop()


@contextlib.contextmanager
def device(spec):
    """Device scope.  `spec` may be a device string or a placement function
    (e.g. `train.replica_device_setter(...)`).  Placement is recorded on
    Variables (`.placement`); compute runs on this process's accelerator."""
    g = get_default_graph()
    g._devices.append(spec)
    try:
        yield spec
    finally:
        g._devices.pop()


def _current_placement(op_type: str, name: str, numel: int) -> Optional[str]:
    g = get_default_graph()
    for spec in reversed(g._devices):
        if callable(spec):
            return spec(_PlacementQuery(op_type, name, numel))
        if spec:
            return str(spec)
    return None


class _PlacementQuery:
    def __init__(self, op_type, name, numel):
        self.type = op_type
        self.name = name
        self.numel = numel
        self.device = ""


# ----------------------------------------------------------------------- tensors
_LOWER_OPS = {"add": "Add", "sub": "Sub", "mul": "Mul", "truediv": "RealDiv", "pow": "Pow", "neg": "Neg",
              "strided_slice": "StridedSlice", "transpose": "Transpose", "concat": "ConcatV2", "stack": "Pack",
              "zeros_like": "ZerosLike", "ones_like": "OnesLike", "clip_by_value": "ClipByValue",
              "gradients": "Gradients", "init": "NoOp", "init_local": "NoOp", "group_deps": "NoOp"}


def _op_type_from_name(name: str) -> str:
    """TF op type for a node built without an explicit one: the
    constructor's default name ("MatMul", "Sigmoid", ...) is the type."""
    base = name.rsplit("/", 1)[-1]
    if base in _LOWER_OPS:
        return _LOWER_OPS[base]
    return base[:1].upper() + base[1:] if base else "Identity"


class RunContext:
    def __init__(self, feeds: Dict[Any, Any], device: torch.device):
        self.feeds = feeds
        self.device = device
        self.memo: Dict[int, Any] = {}
        self.state: Dict[str, Any] = {}

    def eval(self, x):
        if isinstance(x, Tensor):
            k = id(x)
            if k not in self.memo:
                self.memo[k] = x._eval(self)
            return self.memo[k]
        if isinstance(x, (list, tuple)):
            if x and not any(isinstance(v, (Tensor, list, tuple, str, bytes, torch.Tensor, np.ndarray))
                             for v in x):
                return _to_tensor(list(x), self.device)     # python numbers -> constant tensor
            return type(x)(self.eval(v) for v in x)
        return _to_tensor(x, self.device)


def _to_tensor(x, dev, dtype=None):
    if isinstance(x, torch.Tensor):
        t = x.to(dev)
    elif isinstance(x, np.ndarray):
        t = torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    elif isinstance(x, (bytes, str)):
        return x
    elif isinstance(x, (list, tuple)) and x and all(isinstance(v, (bytes, str)) for v in x):
        return list(x)                      # string tensors stay host-side lists
    else:
        t = torch.tensor(x, device=dev)
    if t.dtype == torch.float64:
        t = t.float()
    if dtype is not None and dtype != string:
        t = t.to(dtype)
    return t


class Tensor:
    """Deferred value: fn(*inputs) evaluated inside Session.run."""

    _is_op = False
    _pre_run = None      # async train ops: a hook pulling the ps variables (compat/train.py)
    _lowering = None     # train ops: what compat/lowering.py may replace

    def __init__(self, fn: Callable, inputs: Sequence[Any] = (), name: str = "Tensor", dtype=None,
                 shape=None, op_type: Optional[str] = None, attrs: Optional[Dict[str, Any]] = None):
        g = get_default_graph()
        self.fn = fn
        self.inputs = list(inputs)
        self.name = g.unique_name(name) + ":0"
        self.dtype = dtype
        self.shape = shape
        self.op = self
        self.op_type = op_type or _op_type_from_name(name)   # TF op type for GraphDef / graph rewrites
        self.attrs = attrs or {}
        g._nodes.append(self)

    def _eval(self, ctx: RunContext):
        vals = [ctx.eval(i) for i in self.inputs]
        return self.fn(*vals)

    # arithmetic ----------------------------------------------------------
    # reflected forms keep TF's operand order (x - y with x a constant)
    def __add__(self, o): return Tensor(lambda a, b: a + b, [self, o], "add", op_type="Add")
    def __radd__(self, o): return Tensor(lambda a, b: a + b, [o, self], "add", op_type="Add")
    def __sub__(self, o): return Tensor(lambda a, b: a - b, [self, o], "sub", op_type="Sub")
    def __rsub__(self, o): return Tensor(lambda a, b: a - b, [o, self], "sub", op_type="Sub")
    def __mul__(self, o): return Tensor(lambda a, b: a * b, [self, o], "mul", op_type="Mul")
    def __rmul__(self, o): return Tensor(lambda a, b: a * b, [o, self], "mul", op_type="Mul")
    def __truediv__(self, o): return Tensor(lambda a, b: a / b, [self, o], "truediv", op_type="RealDiv")
    def __rtruediv__(self, o): return Tensor(lambda a, b: a / b, [o, self], "truediv", op_type="RealDiv")
    def __pow__(self, o): return Tensor(lambda a, b: a ** b, [self, o], "pow", op_type="Pow")
    def __neg__(self): return Tensor(lambda a: -a, [self], "Neg", op_type="Neg")
    def __matmul__(self, o): return matmul(self, o)
    def __getitem__(self, idx): return Tensor(lambda a: a[idx], [self], "strided_slice", op_type="StridedSlice")

    def eval(self, session=None, feed_dict=None):
        from .session import get_default_session

        sess = session or get_default_session()
        return sess.run(self, feed_dict=feed_dict)

    def get_shape(self):
        return self.shape

    def set_shape(self, shape):
        """Static shape annotation; checked against the value at run time."""
        self.shape = list(shape)
        inner = self._eval

        def checked(ctx, inner=inner, shape=tuple(shape)):
            v = inner(ctx)
            vs = tuple(getattr(v, "shape", ()))
            if len(vs) != len(shape) or any(a is not None and a != b for a, b in zip(shape, vs)):
                raise ValueError(f"{self.name}: value shape {vs} incompatible with set_shape {list(shape)}")
            return v
        self._eval = checked

    def __repr__(self):
        return f"<dtf Tensor {self.name}>"


class Operation(Tensor):
    """A node run for its side effect; Session.run returns None for it."""

    _is_op = True

    def __init__(self, fn: Callable, inputs: Sequence[Any] = (), name: str = "Op", op_type: Optional[str] = None):
        super().__init__(fn, inputs, name, op_type=op_type or ("NoOp" if not inputs else None))

    def run(self, session=None, feed_dict=None):
        from .session import get_default_session

        (session or get_default_session()).run(self, feed_dict=feed_dict)


def group(*ops, name="group_deps") -> Operation:
    flat = []
    for o in ops:
        flat.extend(o if isinstance(o, (list, tuple)) else [o])
    return Operation(lambda *a: None, flat, name, op_type="NoOp")


def no_op(name="NoOp") -> Operation:
    return Operation(lambda: None, [], name, op_type="NoOp")


def constant(value, dtype=None, shape=None, name="Const") -> Tensor:
    def f():
        t = _to_tensor(value, get_default_graph().device, dtype)
        return t.reshape(shape) if shape is not None and isinstance(t, torch.Tensor) else t
    return Tensor(f, [], name, dtype=dtype, shape=shape, op_type="Const", attrs={"value": value})


class Placeholder(Tensor):
    def __init__(self, dtype=float32, shape=None, name="Placeholder"):
        super().__init__(None, [], name, dtype=dtype, shape=shape, op_type="Placeholder")

    def _eval(self, ctx: RunContext):
        for key in (self, self.name, self.name[:-2]):
            try:
                if key in ctx.feeds:
                    return _to_tensor(ctx.feeds[key], ctx.device, self.dtype)
            except TypeError:
                continue
        raise KeyError(f"You must feed a value for placeholder {self.name}")


def placeholder(dtype=float32, shape=None, name="Placeholder") -> Placeholder:
    return Placeholder(dtype, shape, name)


# ----------------------------------------------------------------------- variables
class Variable(Tensor):
    """TF-style variable: named, initialised by an initializer op, placed per
    the device scope (replica_device_setter records ps/worker placement)."""

    def __init__(self, initial_value=None, trainable: bool = True, name: Optional[str] = None,
                 dtype=None, collections=None, _full_name: Optional[str] = None, partitioner=None):
        g = get_default_graph()
        self._init_value = initial_value
        base = _full_name or g.unique_name(name or "Variable")
        if self._become_partitioned(base, initial_value, trainable, dtype, collections, partitioner):
            return
        self.fn = None
        self.inputs = []
        self.name = base + ":0"
        self.op = self
        self.op_type, self.attrs = "VariableV2", {}
        g._nodes.append(self)
        self.trainable = trainable
        init = self._materialize_initial()
        if dtype is not None:
            init = init.to(dtype)
        self.dtype = init.dtype
        self.shape = tuple(init.shape)
        cached = self.__dict__.pop("_placement_cache", None)
        self.placement = cached[0] if cached else _current_placement("VariableV2", base, init.numel())
        self.value = torch.nn.Parameter(init.to(g.device).clone(), requires_grad=trainable and init.is_floating_point())
        self.initialized = False
        self.initializer = Operation(lambda: self._initialize(), [], base + "/Assign", op_type="Assign")
        self.initializer.name = base + "/Assign:0"          # absolute, like the variable's own name
        cols = collections or ([GLOBAL_VARIABLES] + ([TRAINABLE_VARIABLES] if trainable else []))
        for c in cols:
            g.add_to_collection(c, self)
        g._vars_by_name[base] = self

    def _become_partitioned(self, base, iv, trainable, dtype, collections, partitioner) -> bool:
        from . import partitioned as P

        shape = getattr(iv, "_shape", None)
        spec = getattr(iv, "_init_spec", None)
        if shape is None or spec is None or len(shape) not in (1, 2):
            return False
        if dtype is not None and dtype not in (float32, torch.float32):
            return False
        placement = _current_placement("VariableV2", base, int(np.prod(shape)))
        self._placement_cache = (placement,)
        on_ps = bool(placement) and "/job:ps" in str(placement)
        if partitioner is None and not (on_ps and shape[0] >= P.shard_min_rows()):
            return False
        self.__class__ = P.PartitionedVariable
        P.PartitionedVariable.__init__(self, base, shape, spec, trainable, collections, partitioner, placement)
        return True

    def _materialize_initial(self) -> torch.Tensor:
        iv = self._init_value
        if callable(iv) and not isinstance(iv, Tensor):
            iv = iv()
        if isinstance(iv, Tensor):
            ctx = RunContext({}, torch.device("cpu"))
            iv = ctx.eval(iv)
        if not isinstance(iv, torch.Tensor):
            iv = torch.as_tensor(np.asarray(iv))
            if iv.dtype == torch.float64:
                iv = iv.float()
        return iv.detach().cpu()

    def _initialize(self):
        with torch.no_grad():
            self.value.data.copy_(self._materialize_initial().to(self.value.device, self.value.dtype))
        self.initialized = True

    def _eval(self, ctx: RunContext):
        return self.value

    @property
    def op_name(self) -> str:
        return self.name[:-2]

    def assign(self, value) -> Operation:
        def f(_ref, v):
            with torch.no_grad():
                self.value.data.copy_(torch.as_tensor(v).to(self.value.device, self.value.dtype))
            return self.value
        return Operation(f, [self, value], self.op_name + "/Assign", op_type="Assign")

    def assign_add(self, delta) -> Operation:
        def f(_ref, d):
            with torch.no_grad():
                self.value.data.add_(torch.as_tensor(d).to(self.value.device, self.value.dtype))
            return self.value
        return Operation(f, [self, delta], self.op_name + "/AssignAdd", op_type="AssignAdd")

    def load(self, value, session=None):
        from . import resident
        resident.quiesce_all()         # a resident engine holds this graph's weights in registers
        with torch.no_grad():
            self.value.data.copy_(torch.as_tensor(np.asarray(value)).to(self.value.device, self.value.dtype))

    def read_value(self):
        return self.value.detach()

    def numpy(self):
        return self.value.detach().cpu().numpy()

    def __repr__(self):
        return f"<dtf Variable '{self.name}' shape={self.shape} dtype={self.dtype}>"


# initializers ---------------------------------------------------------------
def _gen(seed):
    g = torch.Generator()
    if seed is None:
        seed = get_default_graph().next_seed()
    if seed is None:
        g.seed()
    else:
        g.manual_seed(int(seed))
    return g


def _spec(fn, shape, kind, a, b, seed):
    fn._init_spec = (kind, a, b, seed)
    fn._shape = tuple(int(s) for s in shape)
    return fn


def random_normal(shape, mean=0.0, stddev=1.0, dtype=float32, seed=None, name="random_normal"):
    if seed is None:
        seed = get_default_graph().next_seed()
    gen = _gen(seed)
    shape = tuple(int(s) for s in shape)
    return _spec(lambda: (torch.randn(shape, generator=gen, dtype=torch.float32) * stddev + mean).to(dtype),
                 shape, "normal", mean, stddev, seed)


def truncated_normal(shape, mean=0.0, stddev=1.0, dtype=float32, seed=None, name="truncated_normal"):
    gen = _gen(seed)
    shape = tuple(int(s) for s in shape)

    def f():
        t = torch.randn(shape, generator=gen)
        while True:
            bad = t.abs() > 2
            if not bad.any():
                break
            t[bad] = torch.randn(int(bad.sum()), generator=gen)
        return (t * stddev + mean).to(dtype)
    return f


def zeros(shape, dtype=float32, name="zeros"):
    return _spec(lambda: torch.zeros(tuple(int(s) for s in shape), dtype=dtype), shape, "const", 0.0, 0, 0)


def ones(shape, dtype=float32, name="ones"):
    return _spec(lambda: torch.ones(tuple(int(s) for s in shape), dtype=dtype), shape, "const", 1.0, 0, 0)


def random_uniform(shape, minval=0.0, maxval=1.0, dtype=float32, seed=None, name="random_uniform"):
    gen = _gen(seed)
    return lambda: (torch.rand(tuple(int(s) for s in shape), generator=gen) * (maxval - minval) + minval).to(dtype)


class constant_initializer:
    def __init__(self, value=0.0, dtype=float32):
        self.value = value
        self.dtype = dtype

    def __call__(self, shape, dtype=None):
        return torch.full(tuple(int(s) for s in shape), float(self.value), dtype=dtype or torch.float32)


class random_normal_initializer:
    def __init__(self, mean=0.0, stddev=1.0, seed=None, dtype=float32):
        self.mean, self.stddev, self.seed = mean, stddev, seed

    def __call__(self, shape, dtype=None):
        return random_normal(shape, self.mean, self.stddev, dtype or float32, self.seed)()


class truncated_normal_initializer(random_normal_initializer):
    def __call__(self, shape, dtype=None):
        return truncated_normal(shape, self.mean, self.stddev, dtype or float32, self.seed)()


class zeros_initializer:
    def __init__(self, dtype=float32):
        self.dtype = dtype

    def __call__(self, shape, dtype=None):
        return torch.zeros(tuple(int(s) for s in shape), dtype=dtype or torch.float32)


class glorot_uniform_initializer:
    def __init__(self, seed=None, dtype=float32):
        self.seed = seed

    def __call__(self, shape, dtype=None):
        fan_in, fan_out = (shape[0], shape[-1]) if len(shape) >= 2 else (shape[0], shape[0])
        lim = (6.0 / (fan_in + fan_out)) ** 0.5
        return random_uniform(shape, -lim, lim, seed=self.seed)()


def get_variable(name, shape=None, dtype=float32, initializer=None, trainable=True, collections=None,
                 partitioner=None) -> Variable:
    """tf.get_variable: honours variable_scope (names) and reuse.  Default
    initializer is glorot-uniform as in TF; `constant_initializer(0)` with no
    dtype yields float32 (the reference's float32 global_step, A5)."""
    g = get_default_graph()
    full = "/".join(g._var_scope + [name]) if g._var_scope else name
    if full in g._vars_by_name:
        if g._var_reuse and g._var_reuse[-1]:
            return g._vars_by_name[full]
        raise ValueError(f"Variable {full} already exists, disallowed. Did you mean to set reuse=True?")
    init = initializer if initializer is not None else glorot_uniform_initializer()
    shp = tuple(int(s) for s in (shape or ()))
    iv = (lambda: init(shp, dtype)) if callable(init) else init
    if callable(iv):
        if isinstance(init, random_normal_initializer) and not isinstance(init, truncated_normal_initializer):
            seed = init.seed if init.seed is not None else g.next_seed()
            iv = _spec(iv, shp, "normal", init.mean, init.stddev, seed)
        elif isinstance(init, (constant_initializer, zeros_initializer)):
            iv = _spec(iv, shp, "const", float(getattr(init, "value", 0.0)), 0, 0)
    v = Variable(iv, trainable=trainable, dtype=dtype, collections=collections, _full_name=full,
                 partitioner=partitioner)
    g._names[full] = g._names.get(full, 0) + 1
    return v


def global_variables():
    return get_default_graph().get_collection(GLOBAL_VARIABLES)


def all_variables():
    return global_variables()


def trainable_variables():
    return get_default_graph().get_collection(TRAINABLE_VARIABLES)


def local_variables():
    return get_default_graph().get_collection(LOCAL_VARIABLES)


def variables_initializer(var_list, name="init") -> Operation:
    return Operation(lambda: [v._initialize() for v in var_list], [], name)


def global_variables_initializer() -> Operation:
    return Operation(lambda: [v._initialize() for v in global_variables()], [], "init")


initialize_all_variables = global_variables_initializer


def local_variables_initializer() -> Operation:
    return Operation(lambda: [v._initialize() for v in local_variables()], [], "init_local")


def report_uninitialized_variables(var_list=None):
    vs = var_list if var_list is not None else global_variables()
    return [v.name for v in vs if not v.initialized]


# ----------------------------------------------------------------------- math ops
def _binary(fn, name):
    def op(a, b, name=None):
        return Tensor(fn, [a, b], name or op_name, op_type=op_name)
    op_name = name
    return op


add = _binary(lambda a, b: a + b, "Add")
subtract = _binary(lambda a, b: a - b, "Sub")
sub = subtract
multiply = _binary(lambda a, b: a * b, "Mul")
mul = multiply
divide = _binary(lambda a, b: a / b, "RealDiv")
div = divide
truediv = divide
maximum = _binary(torch.maximum, "Maximum")
minimum = _binary(torch.minimum, "Minimum")
pow = _binary(lambda a, b: a ** b, "Pow")  # noqa: A001


def matmul(a, b, transpose_a=False, transpose_b=False, name="MatMul") -> Tensor:
    def f(x, y):
        # fp32 stays fp32 (the reference graph's precision): the eager path is
        # a plain library GEMM; the matched training graph runs on the
        # exact-fp32 MFMA kernels of compat/lowering.py instead
        x = x.t() if transpose_a else x
        y = y.t() if transpose_b else y
        return x @ y
    return Tensor(f, [a, b], name, op_type="MatMul",
                  attrs={"transpose_a": bool(transpose_a), "transpose_b": bool(transpose_b)})


def _unary(fn, name):
    def op(x, name=None):
        return Tensor(fn, [x], name or op_name, op_type=op_name)
    op_name = name
    return op


log = _unary(torch.log, "Log")
exp = _unary(torch.exp, "Exp")
sqrt = _unary(torch.sqrt, "Sqrt")
square = _unary(torch.square, "Square")
abs = _unary(torch.abs, "Abs")  # noqa: A001
negative = _unary(torch.neg, "Neg")
sigmoid = _unary(torch.sigmoid, "Sigmoid")
tanh = _unary(torch.tanh, "Tanh")
sin = _unary(torch.sin, "Sin")
cos = _unary(torch.cos, "Cos")
identity = _unary(lambda x: x, "Identity")
stop_gradient = _unary(lambda x: x.detach(), "StopGradient")


def _axes(reduction_indices, axis):
    ax = axis if axis is not None else reduction_indices
    if ax is None:
        return None
    return tuple(ax) if isinstance(ax, (list, tuple)) else (ax,)


def reduce_mean(x, axis=None, keep_dims=False, reduction_indices=None, name="Mean", keepdims=None):
    kd = keep_dims if keepdims is None else keepdims
    ax = _axes(reduction_indices, axis)
    return Tensor(lambda t: t.float().mean() if ax is None else t.float().mean(dim=ax, keepdim=kd), [x], name,
                  op_type="Mean", attrs={"axis": ax, "keep_dims": bool(kd)})


def reduce_sum(x, axis=None, keep_dims=False, reduction_indices=None, name="Sum", keepdims=None):
    kd = keep_dims if keepdims is None else keepdims
    ax = _axes(reduction_indices, axis)
    return Tensor(lambda t: t.sum() if ax is None else t.sum(dim=ax, keepdim=kd), [x], name,
                  op_type="Sum", attrs={"axis": ax, "keep_dims": bool(kd)})


def reduce_max(x, axis=None, keep_dims=False, reduction_indices=None, name="Max"):
    ax = _axes(reduction_indices, axis)
    return Tensor(lambda t: t.max() if ax is None else t.amax(dim=ax, keepdim=keep_dims), [x], name,
                  op_type="Max", attrs={"axis": ax, "keep_dims": bool(keep_dims)})


def argmax(x, axis=None, dimension=None, name="ArgMax"):
    ax = axis if axis is not None else (dimension if dimension is not None else 0)
    return Tensor(lambda t: t.argmax(dim=ax), [x], name, op_type="ArgMax", attrs={"axis": ax})


def argmin(x, axis=None, dimension=None, name="ArgMin"):
    ax = axis if axis is not None else (dimension if dimension is not None else 0)
    return Tensor(lambda t: t.argmin(dim=ax), [x], name, op_type="ArgMin", attrs={"axis": ax})


def equal(a, b, name="Equal"):
    return Tensor(lambda x, y: x == y, [a, b], name, op_type="Equal")


def cast(x, dtype, name="Cast"):
    return Tensor(lambda t: t.to(dtype), [x], name, dtype=dtype, op_type="Cast", attrs={"DstT": dtype})


def reshape(x, shape, name="Reshape"):
    return Tensor(lambda t: t.reshape(tuple(shape)), [x], name, op_type="Reshape", attrs={"shape": list(shape)})


def transpose(x, perm=None, name="transpose"):
    return Tensor(lambda t: t.permute(*perm) if perm is not None else t.t(), [x], name, op_type="Transpose",
                  attrs={"perm": None if perm is None else list(perm)})


def concat(values, axis, name="concat"):
    return Tensor(lambda *ts: torch.cat(ts, dim=axis), list(values), name)


def stack(values, axis=0, name="stack"):
    return Tensor(lambda *ts: torch.stack(ts, dim=axis), list(values), name)


def shape(x, name="Shape"):
    return Tensor(lambda t: torch.tensor(list(t.shape)), [x], name)


def size(x, name="Size"):
    return Tensor(lambda t: torch.tensor(t.numel()), [x], name)


def zeros_like(x, name="zeros_like"):
    return Tensor(torch.zeros_like, [x], name)


def ones_like(x, name="ones_like"):
    return Tensor(torch.ones_like, [x], name)


def clip_by_value(x, lo, hi, name="clip_by_value"):
    return Tensor(lambda t, a, b: torch.clamp(t, a, b), [x, lo, hi], name)


def convert_to_tensor(x, dtype=None, name="Const"):
    return x if isinstance(x, Tensor) else constant(x, dtype=dtype, name=name)


def dynamic_partition(data, partitions, num_partitions, name="DynamicPartition"):
    """Returns a list of tensors: data[partitions == i] (input_pipeline.py:30)."""
    outs = []
    for i in range(num_partitions):
        def f(d, p, i=i):
            if isinstance(d, (list, tuple)):
                return [x for x, q in zip(d, p.tolist()) if q == i]
            if isinstance(d, np.ndarray):
                return d[p.cpu().numpy() == i]
            return d[p == i]
        outs.append(Tensor(f, [data, partitions], f"{name}_{i}"))
    return outs
