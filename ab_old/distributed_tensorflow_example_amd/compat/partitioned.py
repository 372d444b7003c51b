"""PS-placed embedding variables as row-sharded GPU tables (BASELINE config #5).

Reference: `with tf.device(replica_device_setter(cluster=...))` puts
`W = tf.Variable(tf.random_normal([F, 1]))` (F up to 1e9) on /job:ps/task:0
and `embedding_lookup_sparse(W, ...)` pulls only the touched rows over gRPC
(lr2.py:359-390).  Under synchronous data parallelism a dense replica of such
a table per GPU plus a dense all-reduce of its gradient would be absurd, so
the compat layer turns it into a `PartitionedVariable`:

* created when a variable gets a `partitioner=` (tf.fixed_size_partitioner /
  min_max_variable_partitioner / shard_across_workers), or when it is placed
  on a ps task and has >= DTF_SHARD_MIN_ROWS rows (default 1M);
* storage: one shard per worker GPU (parallel.sharded_embedding) -- the ps
  role is spread over all workers, the shard count follows the world size;
* `embedding_lookup(_sparse)` on it runs the all-to-all lookup + CSR bag
  kernel; the optimizer applies the IndexedSlices-style gradient at the
  owners (sparse SGD / ScatterSub), with the 1/W sync-average folded in;
* checkpoints hold the TF PartitionedVariable layout (full-name entry with
  TensorSliceProto slices + one EncodeTensorNameSlice entry per contiguous
  partition; the partitioner's shard count, else one per worker), written in
  parallel into one multi-shard bundle;
* dense use (e.g. matmul on the whole table) gathers the full table with a
  warning -- supported for small tables / tests only.
"""
from __future__ import annotations

import os
import warnings
from typing import Optional

import numpy as np
import torch

from ..parallel import world as _worldmod
from ..parallel.sharded_embedding import ShardedEmbedding
from .graph import (GLOBAL_VARIABLES, TRAINABLE_VARIABLES, RunContext, Tensor, Variable, get_default_graph)

def shard_min_rows() -> int:
    return int(os.environ.get("DTF_SHARD_MIN_ROWS", 1 << 20))


class _Partitioner:
    def __init__(self, num_shards=None, kind="fixed"):
        self.num_shards, self.kind = num_shards, kind

    def __call__(self, shape, dtype=None):   # TF partitioners are callables
        return [self.num_shards or 1] + [1] * (len(shape) - 1)


def fixed_size_partitioner(num_shards, axis=0):
    return _Partitioner(int(num_shards), "fixed")


def min_max_variable_partitioner(max_partitions=1, axis=0, min_slice_size=256 << 10, bytes_per_string_element=16):
    return _Partitioner(int(max_partitions), "min_max")


def variable_axis_size_partitioner(max_shard_bytes, axis=0, bytes_per_string_element=16, max_shards=None):
    return _Partitioner(max_shards, "axis_size")


def shard_across_workers():
    return _Partitioner(None, "workers")


def _world():
    w = _worldmod._WORLD
    return w if w is not None else _worldmod.World(device=get_default_graph().device)


class PartitionedVariable(Variable):
    """A [rows, dim] variable stored as one ShardedEmbedding shard per worker."""

    is_partitioned = True

    def __init__(self, full_name: str, shape, init_spec, trainable=True, collections=None, partitioner=None,
                 placement=None):
        g = get_default_graph()
        self.fn = None
        self.inputs = []
        self.name = full_name + ":0"
        self.op = self
        self.op_type, self.attrs = "VariableV2", {}
        g._nodes.append(self)
        self.trainable = trainable
        self.dtype = torch.float32
        self.shape = tuple(int(s) for s in shape)
        if len(self.shape) not in (1, 2):
            raise ValueError("partitioned variables must be [rows] or [rows, dim]")
        self.rows = self.shape[0]
        self.dim = self.shape[1] if len(self.shape) == 2 else 1
        self.placement = placement
        self.partitioner = partitioner
        kind, a, b, seed = init_spec
        seed = 0 if seed is None else int(seed)       # must agree across ranks without a graph seed
        self._spec = init_spec = (kind, a, b, seed)
        self.world = _world()
        self.table = ShardedEmbedding(self.rows, self.dim, self.world, init_std=b if kind == "normal" else 1.0,
                                      seed=seed, device=g.device, name=full_name, zero_init=(kind == "const"))
        self._post_init()
        self.initialized = False
        from .graph import Operation

        self.initializer = Operation(lambda: self._initialize(), [], full_name + "/Assign", op_type="Assign")
        self.initializer.name = full_name + "/Assign:0"
        cols = collections or ([GLOBAL_VARIABLES] + ([TRAINABLE_VARIABLES] if trainable else []))
        for c in cols:
            g.add_to_collection(c, self)
        g._vars_by_name[full_name] = self

    def _post_init(self):
        kind, a, b, seed = self._spec
        with torch.no_grad():
            if kind == "normal" and a:
                self.table.local.add_(a)
            elif kind == "const":
                self.table.local.fill_(float(a))
            elif kind == "value":
                full = torch.as_tensor(np.asarray(a), dtype=torch.float32).reshape(self.rows, self.dim)
                self.table.load_full(full)

    def _initialize(self):
        kind, a, b, seed = self._spec
        if kind == "normal":
            fresh = ShardedEmbedding(self.rows, self.dim, self.world, init_std=b, seed=seed,
                                     device=self.table.device, name=self.table.name)
            with torch.no_grad():
                self.table.local.copy_(fresh.local)
        self._post_init()
        self.initialized = True

    # -- storage seen by Saver / broadcast: the local shard -------------------
    @property
    def value(self):
        return self.table.local

    @property
    def part_name(self) -> str:
        return self.table.shard_name()

    def _eval(self, ctx: RunContext):
        warnings.warn(f"dense use of partitioned variable {self.name}: gathering {self.rows} rows")
        full = self.table.full_table()
        return full if len(self.shape) == 2 else full.reshape(-1)

    def load(self, value, session=None):
        self.table.load_full(torch.as_tensor(np.asarray(value), dtype=torch.float32).reshape(self.rows, self.dim))

    def numpy(self):
        return self.table.full_table().cpu().numpy().reshape(self.shape)

    def __repr__(self):
        return f"<dtf PartitionedVariable '{self.name}' shape={self.shape} shards={self.world.world_size}>"


class PartitionedSlot:
    """An optimizer slot of a partitioned variable (`<var>/Adagrad`,
    `<var>/Adam_1`, ...): sharded exactly like the table, checkpointed in the
    same TF slice layout, not trainable."""

    is_partitioned = True
    op_type, attrs = "VariableV2", {}

    def __init__(self, pv: PartitionedVariable, slot: str):
        self.pv, self.slot = pv, slot
        self.name = f"{pv.name[:-2]}/{slot}:0"
        self.shape, self.rows, self.dim, self.dtype = pv.shape, pv.rows, pv.dim, torch.float32
        self.partitioner, self.world = pv.partitioner, pv.world
        self.trainable = False
        self.initialized = True
        self.placement = pv.placement
        # the value the optimizer gives the slot (Adagrad: initial_accumulator_value, RMSProp ms: 1)
        self.init = {"Adagrad": float(pv.table.opt_hp.get("initial_accumulator_value", 0.1)),
                     "RMSProp": 1.0}.get(slot, 0.0)

    @property
    def table(self):
        return self.pv.table.slot_view(self.slot)

    @property
    def value(self):
        return self.pv.table.slots[self.slot]

    def _initialize(self):
        with torch.no_grad():
            self.value.fill_(self.init)

    def __repr__(self):
        return f"<dtf PartitionedSlot '{self.name}' shape={self.shape}>"


def init_spec_of(initial_value, graph_seed_fn) -> Optional[tuple]:
    """('normal', mean, std, seed) | ('const', v, 0, 0) | None for an initial value."""
    spec = getattr(initial_value, "_init_spec", None)
    if spec is not None:
        kind, a, b, seed = spec
        if seed is None:
            seed = graph_seed_fn()
        return (kind, a, b, 0 if seed is None else int(seed))
    return None


def lookup_sparse(ctx: RunContext, pv: PartitionedVariable, sp_ids, sp_w, combiner: str):
    """Bag lookup on the sharded table; records (pv, state) for the optimizer."""
    from .sparse import SparseTensor

    offsets, ids, vals = SparseTensor.to_csr(sp_ids, sp_w)
    dev = pv.table.device
    out, st = pv.table.bag_forward(ids.to(dev), offsets.to(dev), None if vals is None else vals.to(dev).float(),
                                   combiner)
    ctx.state.setdefault("pv_lookups", []).append((pv, st))
    return out if len(pv.shape) == 2 else out


def lookup_dense(ctx: RunContext, pv: PartitionedVariable, ids):
    ids = ids.reshape(-1).long().to(pv.table.device)
    rows, lctx = pv.table.lookup(ids)
    rows = rows.detach().requires_grad_(True)
    ctx.state.setdefault("pv_lookups", []).append((pv, (rows, lctx)))
    out = rows[lctx.inverse]
    return out if len(pv.shape) == 2 else out.reshape(-1)
