"""tf.SparseTensor (COO) and its CSR view for the embedding-bag kernels.

lr2.py:372-378 feeds `SparseTensor(shape=[F, B], indices=[[row, fid]...],
values=fids|fvals)`; TF's embedding_lookup_sparse only uses indices[:, 0] as
the (sorted) segment id and emits max(segment)+1 rows -- the odd [F, B] shape
is ignored, and so it is here.
"""
from __future__ import annotations

import numpy as np
import torch

from .graph import Tensor, _to_tensor


class SparseTensorValue:
    def __init__(self, indices, values, dense_shape):
        self.indices = indices
        self.values = values
        self.dense_shape = dense_shape


class SparseTensor(Tensor):
    def __init__(self, indices=None, values=None, dense_shape=None, shape=None):
        ds = dense_shape if dense_shape is not None else shape
        super().__init__(lambda i, v, s: SparseTensorValue(i, v, s), [indices, values, ds], "SparseTensor")
        self.indices = indices
        self.values = values
        self.dense_shape = ds

    @staticmethod
    def to_csr(ids_sp: SparseTensorValue, w_sp: SparseTensorValue = None):
        idx = ids_sp.indices
        idx = idx if isinstance(idx, torch.Tensor) else torch.as_tensor(np.asarray(idx))
        ids = ids_sp.values
        ids = ids if isinstance(ids, torch.Tensor) else torch.as_tensor(np.asarray(ids))
        if idx.numel() == 0:
            return torch.zeros(1, dtype=torch.int64), ids.long(), None
        rows = idx.reshape(-1, idx.shape[-1])[:, 0].long().cpu()
        nb = int(rows.max()) + 1
        counts = torch.bincount(rows, minlength=nb)
        offsets = torch.zeros(nb + 1, dtype=torch.int64)
        offsets[1:] = torch.cumsum(counts, 0)
        vals = None
        if w_sp is not None and w_sp is not ids_sp:
            vals = w_sp.values
            vals = vals if isinstance(vals, torch.Tensor) else torch.as_tensor(np.asarray(vals, dtype=np.float32))
        return offsets, ids.long(), vals


def sparse_tensor_to_dense(sp, default_value=0):
    def f(v):
        idx = torch.as_tensor(np.asarray(v.indices)).long()
        vals = torch.as_tensor(np.asarray(v.values))
        shape = [int(s) for s in np.asarray(v.dense_shape)]
        out = torch.full(shape, default_value, dtype=vals.dtype)
        out[tuple(idx.t())] = vals
        return out
    return Tensor(f, [sp], "SparseToDense")
