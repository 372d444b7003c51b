"""TF-format checkpoints (V2 tensor bundle) for compat Variables.

Reference: `tf.train.Saver()` (model_export.py:53) and the Supervisor's
implicit saver (inactive there, no logdir); BASELINE requires the TF
checkpoint format to stay compatible.  Bytes are produced by the native
writer (csrc/runtime/tf_bundle.cpp): `prefix.index` (leveldb table of
BundleEntryProto) + `prefix.data-00000-of-00001` + the text `checkpoint`
state file (`model_checkpoint_path: "model.ckpt-N"`).  Variable names are the
TF names (`weights/Variable_1`, `global_step`, Adam slots `w/Adam`, `w/Adam_1`,
`beta1_power`...).  Only the chief writes; every rank can restore.

Partitioned variables are laid out as TF's Saver writes a PartitionedVariable
(SaveSliceInfo + SaveV2 -> BundleWriter::AddSlice): the full name (`W`)
carries dtype, full shape and a TensorSliceProto per partition, each
partition's bytes sit under `EncodeTensorNameSlice(W, slice)`, and the
partitions are contiguous row ranges as tf.fixed_size_partitioner makes them.
Every rank assembles and writes the partitions it is assigned into its own
data shard; restore accepts any partition count and any writer world size,
or a plain full entry (an unpartitioned TF variable).
"""
from __future__ import annotations

import glob
import os
import re
import time
from typing import Dict, List, Optional

import numpy as np
import torch

from .. import _native

TORCH_TO_TF = {torch.float32: 1, torch.float64: 2, torch.int32: 3, torch.uint8: 4, torch.int16: 5,
               torch.int8: 6, torch.int64: 9, torch.bool: 10, torch.bfloat16: 14, torch.float16: 19}
TF_TO_TORCH = {v: k for k, v in TORCH_TO_TF.items()}
TF_TO_NUMPY = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8, 9: np.int64,
               10: np.bool_, 19: np.float16}


def _np_bytes(t: torch.Tensor):
    t = t.detach().cpu().contiguous()
    dt = TORCH_TO_TF.get(t.dtype)
    if dt is None:
        raise TypeError(f"unsupported dtype {t.dtype}")
    arr = t.view(torch.int16).numpy() if t.dtype == torch.bfloat16 else t.numpy()
    return dt, np.ascontiguousarray(arr).reshape(-1).view(np.uint8)


def write_bundle(prefix: str, tensors: Dict[str, torch.Tensor], shard_id: int = 0, num_shards: int = 1,
                 slices=None):
    """Write {name: tensor} as a TF V2 bundle (names sorted inside the index).

    `slices`: [(full_name, full_shape, extents, tensor)] -- partitions of a
    variable as TF's SaveV2 writes them for SaveSliceInfo specs: the data under
    the EncodeTensorNameSlice key, the slice recorded in the full-name entry.
    `extents` = [(start, length)] per dim (length -1 = the whole dim)."""
    C = _native.load()
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    w = C.BundleWriter(prefix, shard_id, num_shards)
    for name in sorted(tensors):
        dt, buf = _np_bytes(tensors[name])
        w.add(name, dt, list(tensors[name].shape), buf)
    for full_name, full_shape, ext, t in slices or ():
        dt, buf = _np_bytes(t)
        w.add_slice(full_name, dt, [int(x) for x in full_shape], [(int(a), int(b)) for a, b in ext], buf)
    w.finish()


def slice_key(name: str, extents) -> bytes:
    """checkpoint::EncodeTensorNameSlice(name, slice) (OrderedCode bytes)."""
    return _native.load().bundle_slice_key(name, [(int(a), int(b)) for a, b in extents])


def partition_extents(rows: int, num_partitions: int):
    """Row ranges of tf.fixed_size_partitioner(P) on axis 0: the first
    rows % P partitions hold one extra row (variable_scope's
    _get_partitioned_variable slicing)."""
    P = max(1, min(int(num_partitions), int(rows))) if rows else 1
    base, extra = divmod(int(rows), P)
    out, s = [], 0
    for k in range(P):
        n = base + (1 if k < extra else 0)
        out.append((s, n))
        s += n
    return out


def _to_torch(raw, dt, shape) -> torch.Tensor:
    if dt == 14:
        t = torch.from_numpy(np.frombuffer(raw, dtype=np.int16).copy()).view(torch.bfloat16)
    else:
        t = torch.from_numpy(np.frombuffer(raw, dtype=TF_TO_NUMPY[dt]).copy())
    return t.reshape(shape)


def _slice_shape(full_shape, ext):
    return [fs if n < 0 else n for fs, (_, n) in zip(full_shape, ext)]


def read_slice(prefix: str, name: str, extents, entry=None) -> torch.Tensor:
    """One saved slice of a partitioned tensor."""
    C = _native.load()
    e = entry or C.bundle_read_index(prefix)[name]
    raw = C.bundle_read_slice(prefix, name, [(int(a), int(b)) for a, b in extents], True)
    return _to_torch(raw, e["dtype"], _slice_shape(e["shape"], extents))


def iter_slices(prefix: str, name: str, entry=None):
    """(extents, tensor) for every saved slice of `name` -- one slice resident
    at a time, so a partitioned 1e9-row table is restored in pieces."""
    e = entry or read_bundle_index(prefix)[name]
    for ext in e["slices"]:
        yield [tuple(x) for x in ext], read_slice(prefix, name, ext, e)


def read_bundle_index(prefix: str) -> dict:
    return _native.load().bundle_read_index(prefix)


def read_tensor(prefix: str, name: str) -> torch.Tensor:
    """The full tensor `name`; a partitioned (sliced) entry is assembled from
    its slices, as tf.train.NewCheckpointReader does."""
    C = _native.load()
    idx = C.bundle_read_index(prefix)
    if name not in idx:
        raise KeyError(f"{name} not found in checkpoint {prefix}")
    e = idx[name]
    if not e["has_slices"]:
        return _to_torch(C.bundle_read_tensor(prefix, name, True), e["dtype"], e["shape"])
    out = None
    covered = 0
    for ext, t in iter_slices(prefix, name, e):
        if out is None:
            out = torch.empty(list(e["shape"]), dtype=t.dtype)
        sl = tuple(slice(None) if n < 0 else slice(a, a + n) for a, n in ext)
        out[sl] = t
        covered += t.numel()
    if out is None or covered != out.numel():
        raise ValueError(f"slices of {name} in {prefix} do not cover the tensor ({covered} of "
                         f"{0 if out is None else out.numel()} elements)")
    return out


def list_variables(ckpt: str):
    prefix = _resolve(ckpt)
    return [(k, list(v["shape"])) for k, v in sorted(read_bundle_index(prefix).items()) if k]


def load_variable(ckpt: str, name: str) -> np.ndarray:
    return read_tensor(_resolve(ckpt), name).float().numpy() if read_tensor(_resolve(ckpt), name).dtype == torch.bfloat16 \
        else read_tensor(_resolve(ckpt), name).numpy()


class CheckpointReader:
    """tf.train.NewCheckpointReader equivalent."""

    def __init__(self, prefix):
        self.prefix = _resolve(prefix)
        self._idx = read_bundle_index(self.prefix)

    def get_variable_to_shape_map(self):
        return {k: list(v["shape"]) for k, v in self._idx.items() if k}

    def get_variable_to_dtype_map(self):
        return {k: TF_TO_TORCH.get(v["dtype"]) for k, v in self._idx.items() if k}

    def has_tensor(self, name):
        return name in self._idx and name != ""

    def get_tensor(self, name) -> np.ndarray:
        t = read_tensor(self.prefix, name)
        return t.float().numpy() if t.dtype == torch.bfloat16 else t.numpy()


def NewCheckpointReader(prefix):  # noqa: N802 (TF name)
    return CheckpointReader(prefix)


# ----------------------------------------------------------------------- state file
class CheckpointState:
    def __init__(self, model_checkpoint_path: str, all_model_checkpoint_paths: List[str]):
        self.model_checkpoint_path = model_checkpoint_path
        self.all_model_checkpoint_paths = list(all_model_checkpoint_paths)

    def __repr__(self):
        return f"CheckpointState({self.model_checkpoint_path!r}, {self.all_model_checkpoint_paths!r})"


def _state_path(d):
    return os.path.join(d, "checkpoint")


def update_checkpoint_state(save_dir: str, model_checkpoint_path: str, all_model_checkpoint_paths=None,
                            latest_filename: str = "checkpoint"):
    allp = list(all_model_checkpoint_paths or [model_checkpoint_path])
    if model_checkpoint_path not in allp:
        allp.append(model_checkpoint_path)

    def rel(p):
        return os.path.relpath(p, save_dir) if os.path.isabs(p) and os.path.dirname(p) == os.path.abspath(save_dir) else p
    lines = [f'model_checkpoint_path: "{rel(model_checkpoint_path)}"']
    lines += [f'all_model_checkpoint_paths: "{rel(p)}"' for p in allp]
    tmp = os.path.join(save_dir, latest_filename + ".tmp")
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, os.path.join(save_dir, latest_filename))


def get_checkpoint_state(checkpoint_dir: str, latest_filename: str = "checkpoint") -> Optional[CheckpointState]:
    p = os.path.join(checkpoint_dir, latest_filename)
    if not os.path.exists(p):
        return None
    model, allp = None, []
    for line in open(p):
        m = re.match(r'\s*(model_checkpoint_path|all_model_checkpoint_paths)\s*:\s*"(.*)"', line)
        if not m:
            continue
        path = m.group(2)
        if not os.path.isabs(path):
            path = os.path.join(checkpoint_dir, path)
        if m.group(1) == "model_checkpoint_path":
            model = path
        else:
            allp.append(path)
    return CheckpointState(model, allp) if model else None


def checkpoint_exists(prefix: str) -> bool:
    return os.path.exists(prefix + ".index")


def latest_checkpoint(checkpoint_dir: str, latest_filename: str = "checkpoint") -> Optional[str]:
    st = get_checkpoint_state(checkpoint_dir, latest_filename)
    if st and checkpoint_exists(st.model_checkpoint_path):
        return st.model_checkpoint_path
    return None


def _resolve(ckpt: str) -> str:
    if os.path.isdir(ckpt):
        p = latest_checkpoint(ckpt)
        if p is None:
            raise FileNotFoundError(f"no checkpoint in {ckpt}")
        return p
    return ckpt


# ----------------------------------------------------------------------- meta graphs
def export_meta_graph(filename: Optional[str] = None, **kw) -> bytes:
    """tf.train.export_meta_graph: MetaGraphDef bytes of the default graph."""
    from .meta_graph import export_meta_graph_bytes

    b = export_meta_graph_bytes()
    if filename:
        with open(filename, "wb") as f:
            f.write(b)
    return b


def read_meta_graph(filename: str) -> dict:
    """Decoded MetaGraphDef (plain dicts; compat/meta_graph.parse_meta_graph)."""
    from .meta_graph import parse_meta_graph

    with open(filename, "rb") as f:
        return parse_meta_graph(f.read())


# ----------------------------------------------------------------------- Saver
def _num_partitions(v) -> int:
    """Partitions TF would create: the partitioner's shard count, else (PS
    placement / shard_across_workers) one per worker."""
    p = getattr(v, "partitioner", None)
    n = getattr(p, "num_shards", None) if p is not None else None
    return int(n) if n else v.world.world_size


class Saver:
    def __init__(self, var_list=None, max_to_keep: int = 5, keep_checkpoint_every_n_hours: float = 10000.0,
                 sharded: bool = False, name: str = None, restore_sequentially: bool = False,
                 write_version: int = 2, save_relative_paths: bool = False, defer_build=False, **kw):
        self._var_list = var_list
        self.max_to_keep = max_to_keep
        self.keep_every = keep_checkpoint_every_n_hours * 3600.0
        self._last_kept = time.time()
        self._kept: List[str] = []
        self.sharded = sharded

    def _vars(self) -> Dict[str, object]:
        from .graph import global_variables

        vl = self._var_list
        if vl is None:
            vl = global_variables()
        if isinstance(vl, dict):
            return dict(vl)
        out = {}
        for v in vl:
            out[v.name[:-2] if v.name.endswith(":0") else v.name] = v
        return out

    @staticmethod
    def _value(v) -> torch.Tensor:
        if hasattr(v, "value") and isinstance(v.value, torch.Tensor):
            return v.value
        if isinstance(v, torch.Tensor):
            return v
        raise TypeError(f"cannot save {v!r}")

    def save(self, sess=None, save_path: str = "model.ckpt", global_step=None, latest_filename="checkpoint",
             meta_graph_suffix="meta", write_meta_graph=True, write_state=True) -> Optional[str]:
        from ..parallel.world import get_world

        step = global_step
        if step is not None and not isinstance(step, (int, np.integer)):
            step = int(np.asarray(sess.run(step) if hasattr(step, "_eval") else step))
        w = get_world()
        vars_ = self._vars()
        parts = {k: v for k, v in vars_.items() if getattr(v, "is_partitioned", False)}
        if parts and w.world_size > 1 and step is not None:
            # a sharded save is collective: every rank must write the same prefix.
            # Asynchronous workers' global_step copies differ (each saw the shared
            # counter at its own last update): use the latest of them
            step = int(w.host_all_reduce(float(step), "max"))
        prefix = f"{save_path}-{int(step)}" if step is not None else save_path
        tensors = {k: self._value(v) for k, v in vars_.items() if k not in parts}
        if parts:
            # TF layout: full-name entry + one slice entry per fixed_size partition;
            # partition k is assembled (rows gathered from the modulo-sharded
            # storage) on rank k % W, which writes it into its own data shard
            from ..ckpt import gather_partitions

            mine = []
            for name in sorted(parts):
                v = parts[name]
                mine += gather_partitions(v.table, name, list(v.shape), _num_partitions(v), w)
            if w.world_size > 1:
                write_bundle(prefix, tensors if w.rank == 0 else {}, shard_id=w.rank, num_shards=w.world_size,
                             slices=mine)
                w.barrier()
                if w.rank == 0:
                    _native.load().bundle_merge_shard_indexes(prefix, w.world_size, True)
                write_meta_graph = write_meta_graph and w.rank == 0
            else:
                write_bundle(prefix, tensors, slices=mine)
        elif w.rank == 0:
            write_bundle(prefix, tensors)
        if w.rank == 0:
            if write_meta_graph:
                self.export_meta_graph(f"{prefix}.{meta_graph_suffix}")
            d = os.path.dirname(os.path.abspath(prefix))
            self._kept.append(prefix)
            while self.max_to_keep and len(self._kept) > self.max_to_keep:
                old = self._kept.pop(0)
                if time.time() - self._last_kept >= self.keep_every:
                    self._last_kept = time.time()
                    continue
                for f in glob.glob(old + ".*"):
                    try:
                        os.remove(f)
                    except OSError:
                        pass
            if write_state:
                update_checkpoint_state(d, os.path.abspath(prefix), [os.path.abspath(p) for p in self._kept],
                                        latest_filename)
        return prefix

    def restore(self, sess=None, save_path: str = None):
        from . import resident
        resident.quiesce_all()         # restored values must not be overwritten by a resident engine
        prefix = _resolve(save_path)
        idx = read_bundle_index(prefix)
        missing = []
        for name, v in self._vars().items():
            if name not in idx:
                old = _old_modulo_parts(idx, name)
                if old:
                    # this repo's earlier layout: `name/part_k` = the rows r % P == k
                    full = _rebuild_modulo(prefix, name, old)
                    if getattr(v, "is_partitioned", False):
                        v.table.load_full(full.reshape(v.table.num_rows, v.table.dim))
                    else:
                        dst = self._value(v)
                        if full.numel() != dst.numel():
                            raise ValueError(f"shape mismatch for {name}: old-layout parts hold {full.numel()} "
                                             f"values vs {tuple(dst.shape)}")
                        with torch.no_grad():
                            dst.data.copy_(full.reshape(dst.shape).to(dst.device, dst.dtype))
                    if hasattr(v, "initialized"):
                        v.initialized = True
                    continue
                missing.append(name)
                continue
            if getattr(v, "is_partitioned", False):
                # sliced (any partition count, any writer world size) or a plain
                # full entry: each rank keeps the rows it owns
                from ..ckpt import restore_table

                restore_table(prefix, name, v.table, idx[name])
                v.initialized = True
                continue
            t = read_tensor(prefix, name)
            if hasattr(v, "restore_from"):     # derived state (Adam's beta powers -> step counts)
                v.restore_from(t)
                continue
            dst = self._value(v)
            if tuple(t.shape) != tuple(dst.shape):
                raise ValueError(f"shape mismatch for {name}: ckpt {tuple(t.shape)} vs {tuple(dst.shape)}")
            with torch.no_grad():
                dst.data.copy_(t.to(dst.device, dst.dtype))
            if hasattr(v, "initialized"):
                v.initialized = True
        if missing:
            raise KeyError(f"variables not found in checkpoint {prefix}: {missing}")

    def export_meta_graph(self, filename: Optional[str] = None, collection_list=None, as_text=False, **kw) -> bytes:
        """Serialized MetaGraphDef of the default graph (graph_def, this
        saver's SaverDef, the collections) -- what Saver.save writes to
        `prefix.meta`."""
        from .meta_graph import export_meta_graph_bytes

        b = export_meta_graph_bytes(saver=self)
        if filename:
            tmp = filename + ".tmp"
            with open(tmp, "wb") as f:
                f.write(b)
            os.replace(tmp, filename)
        return b

    def recover_last_checkpoints(self, paths):
        self._kept = [p for p in paths if checkpoint_exists(p)]

    @property
    def last_checkpoints(self):
        return list(self._kept)

    def as_saver_def(self):
        return {"version": 2, "max_to_keep": self.max_to_keep}


def _old_modulo_parts(idx, name: str):
    """Keys `name/part_0 .. name/part_{P-1}` of the pre-TF-slice layout (rows
    r % P == k in part k, in row order), or [] if absent / incomplete."""
    keys = [k for k in idx if k.startswith(name + "/part_") and k[len(name) + 6:].isdigit()]
    if not keys:
        return []
    P = len(keys)
    want = [f"{name}/part_{k}" for k in range(P)]
    if sorted(keys) != sorted(want):
        raise KeyError(f"checkpoint has an incomplete old-layout partition set for {name}: {sorted(keys)}")
    return want


def _rebuild_modulo(prefix: str, name: str, keys) -> torch.Tensor:
    """Full [rows, dim] table from the old modulo parts (row r = part r % P, row r // P)."""
    parts = [read_tensor(prefix, k).float() for k in keys]
    P = len(parts)
    dim = 1 if parts[0].dim() == 1 else int(parts[0].shape[1])
    parts = [p.reshape(-1, dim) for p in parts]
    rows = sum(p.shape[0] for p in parts)
    for k, p in enumerate(parts):
        if p.shape[0] != (rows - k + P - 1) // P:
            raise ValueError(f"{name}: old-layout part {k} has {p.shape[0]} rows, expected {(rows - k + P - 1) // P}")
    full = torch.empty((rows, dim), dtype=torch.float32)
    for k, p in enumerate(parts):
        full[k::P] = p
    return full
