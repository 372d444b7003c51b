"""Sparse libsvm input path: parser, CSR batches, DataProvider.

Reference (lr2.py): `Sample.parse_line_libsvm` (:57-67) splits each line in
Python; `format_samples_sparse` (:69-84) builds COO `[[row, fid], ...]` lists;
`LoadDataThread` (:87-155) has N Python threads read strided files through
GFile with per-line Bernoulli sampling, either materialising everything
('all') or pushing raw lines into a TF FIFOQueue forever ('queue');
`DataProvider` (:177-304) shards files per worker (`files[task::workers]`),
shuffles per epoch, yields batches and samples a test subset.

Here the parsing is native C++ (csrc/runtime/libsvm.cpp: one thread per file
group, no GIL, sampling in the parser) and a batch is *CSR* --
(labels [B,1] f32, offsets [B+1] i64, ids [nnz] i64, vals [nnz] f32) -- which
is exactly what the embedding-bag kernel consumes; the COO `sp_indices` of the
reference is derivable (`CSRBatch.coo_indices`).  'queue' mode is the native
`LibsvmStream` (bounded queue of ready CSR batches, looping over the files).
Intentional fix: the reference's queue-mode test sampler reads the *train*
queue (lr2.py:213-217, "should be 'test'"); here it reads the test stream.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import Iterator, List, Optional, Sequence

import numpy as np

from .. import _native
from ..utils import gfile
from ..utils import logging as log


@dataclass
class CSRBatch:
    labels: np.ndarray     # [B, 1] float32
    offsets: np.ndarray    # [B + 1] int64
    ids: np.ndarray        # [nnz] int64
    vals: np.ndarray       # [nnz] float32

    @property
    def size(self) -> int:
        return len(self.offsets) - 1

    @property
    def nnz(self) -> int:
        return len(self.ids)

    def coo_indices(self) -> np.ndarray:
        """[[row, fid], ...] of lr2.py:82-83 (SparseTensor indices)."""
        rows = np.repeat(np.arange(self.size, dtype=np.int64), np.diff(self.offsets))
        return np.stack([rows, self.ids], 1)

    def as_tf_feed(self):
        """(labels, fids, fvals, sp_indices, size) == Sample.format_samples_sparse."""
        return self.labels, self.ids, self.vals, self.coo_indices(), self.size

    def to(self, device):
        import torch

        return (torch.from_numpy(self.labels).to(device, non_blocking=True),
                torch.from_numpy(self.offsets).to(device, non_blocking=True),
                torch.from_numpy(self.ids).to(device, non_blocking=True),
                torch.from_numpy(self.vals).to(device, non_blocking=True))


class CSRData:
    """A materialised CSR sample set with vectorised row gathering."""

    def __init__(self, labels, offsets, ids, vals):
        self.labels = np.asarray(labels, np.float32).reshape(-1)
        self.offsets = np.asarray(offsets, np.int64)
        self.ids = np.asarray(ids, np.int64)
        self.vals = np.asarray(vals, np.float32)

    @staticmethod
    def concat(parts: Sequence["CSRData"]) -> "CSRData":
        parts = [p for p in parts if p is not None and len(p)]
        if not parts:
            return CSRData(np.zeros(0), np.zeros(1, np.int64), np.zeros(0, np.int64), np.zeros(0))
        offs, base = [np.zeros(1, np.int64)], 0
        for p in parts:
            offs.append(p.offsets[1:] + base)
            base += p.offsets[-1]
        return CSRData(np.concatenate([p.labels for p in parts]), np.concatenate(offs),
                       np.concatenate([p.ids for p in parts]), np.concatenate([p.vals for p in parts]))

    def __len__(self):
        return len(self.labels)

    def take(self, rows: np.ndarray) -> CSRBatch:
        rows = np.asarray(rows, np.int64)
        starts, ends = self.offsets[rows], self.offsets[rows + 1]
        lens = ends - starts
        offs = np.zeros(len(rows) + 1, np.int64)
        np.cumsum(lens, out=offs[1:])
        idx = np.repeat(starts - offs[:-1], lens) + np.arange(offs[-1], dtype=np.int64)
        return CSRBatch(self.labels[rows].reshape(-1, 1), offs, self.ids[idx], self.vals[idx])

    def slice(self, s: int, e: int) -> CSRBatch:
        return self.take(np.arange(s, e))


def parse_lines(lines: Sequence[str], sampling_rate: float = 1.0, seed: int = 0) -> CSRData:
    data = "".join(l if l.endswith("\n") else l + "\n" for l in lines).encode()
    y, rp, ids, vals = _native.load().libsvm_parse_bytes(data, sampling_rate, seed)
    return CSRData(y, rp, ids, vals)


def load_files(files: Sequence[str], nthreads: int = 2, sampling_rate: float = 1.0, seed: int = 0) -> CSRData:
    """Parse files (local, file:// or hdfs://) with `nthreads` native threads."""
    C = _native.load()
    local = [gfile.local_path(f) for f in files]
    if all(p is not None for p in local):
        y, rp, ids, vals = C.libsvm_parse_files(list(local), int(nthreads), float(sampling_rate), int(seed))
        return CSRData(y, rp, ids, vals)
    parts = []
    for i, f in enumerate(files):    # remote scheme: stream bytes through GFile
        with gfile.GFile(f, "rb") as fh:
            y, rp, ids, vals = C.libsvm_parse_bytes(fh.read(), float(sampling_rate), int(seed) + i)
        parts.append(CSRData(y, rp, ids, vals))
    return CSRData.concat(parts)


def split_file_list(spec: str, num_workers: int = 1, task_index: int = 0) -> List[str]:
    """`files[task_index::num_workers]` of lr2.py:302-304.  `spec` is a comma
    list, or `@listfile` (one path per line, run.sh / lr2_debug.py:220-224),
    or a glob."""
    spec = spec.strip()
    if spec.startswith("@"):
        with gfile.GFile(spec[1:], "r") as f:
            files = [l.strip() for l in f if l.strip()]
    else:
        files = [f.strip() for f in spec.strip(",").split(",") if f.strip()]
        out = []
        for f in files:
            out.extend(sorted(gfile.Glob(f)) if any(c in f for c in "*?[") else [f])
        files = out
    return files[task_index::num_workers]


class DataProvider:
    """Per-worker sparse data facade with the reference's method names."""

    def __init__(self, num_workers: int, task_index: int, thread_num: int = 2, mode: str = "all",
                 train: str = "", test: str = "", batch_size: int = 500, train_sampling_rate: float = 1.0,
                 test_sampling_rate: float = 1.0, queue_capacity: int = 16, seed: int = 0):
        if mode not in ("all", "queue"):
            raise ValueError("mode must be 'all' or 'queue'")
        self.mode, self.num_workers, self.task_index = mode, num_workers, task_index
        self.thread_num = max(1, int(thread_num))
        self.batch_size = int(batch_size)
        self.train_spec, self.test_spec = train, test
        self.train_rate, self.test_rate = train_sampling_rate, test_sampling_rate
        self.queue_capacity = queue_capacity
        self.rng = np.random.default_rng(seed + task_index)
        self.seed = seed
        self.train_file_list: List[str] = []
        self.test_file_list: List[str] = []
        self.train: Optional[CSRData] = None
        self.test: Optional[CSRData] = None
        self._order = None
        self._streams = {}

    # ------------------------------------------------------------ lifecycle
    def init(self, sess=None):
        self.train_file_list = split_file_list(self.train_spec, self.num_workers, self.task_index) \
            if self.train_spec else []
        self.test_file_list = split_file_list(self.test_spec, self.num_workers, self.task_index) \
            if self.test_spec else []
        return self

    def LoadData(self):  # noqa: N802 (reference name)
        t0 = time.time()
        if self.mode == "all":
            self.train = load_files(self.train_file_list, self.thread_num, self.train_rate, self.seed)
            self.test = load_files(self.test_file_list, self.thread_num, self.test_rate, self.seed + 7919)
            self._order = np.arange(len(self.train))
            log.info(f"[worker:{self.task_index}] loaded {len(self.train)} train / {len(self.test)} test "
                     f"samples from {len(self.train_file_list)}+{len(self.test_file_list)} files "
                     f"in {time.time() - t0:.2f}s")
        else:
            C = _native.load()
            for kind, files, rate in (("train", self.train_file_list, self.train_rate),
                                      ("test", self.test_file_list, self.test_rate)):
                local = [gfile.local_path(f) or f for f in files]
                if files:
                    self._streams[kind] = C.LibsvmStream(local, self.batch_size, self.thread_num, float(rate),
                                                         True, int(self.queue_capacity), int(self.seed))
        return self

    def close(self):
        for s in self._streams.values():
            s.stop()
        self._streams.clear()

    # ------------------------------------------------------------ accessors
    def GetTrainSamples(self) -> CSRData:  # noqa: N802
        return self.train

    def GetTestSamples(self) -> CSRData:  # noqa: N802
        return self.test

    def Shuffle(self):  # noqa: N802
        if self._order is not None:
            self.rng.shuffle(self._order)

    def NextBatch(self, data_type: str = "train", max_batches: Optional[int] = None) -> Iterator[CSRBatch]:  # noqa: N802
        if self.mode == "all":
            data = self.train if data_type == "train" else self.test
            order = self._order if data_type == "train" else np.arange(len(data))
            n = len(data)
            for k, s in enumerate(range(0, n, self.batch_size)):
                if max_batches is not None and k >= max_batches:
                    return
                yield data.take(order[s:s + self.batch_size])
        else:
            st = self._streams.get(data_type)
            if st is None:
                return
            k = 0
            while max_batches is None or k < max_batches:
                b = st.next(30.0)
                if b is None:
                    return
                y, rp, ids, vals = b
                yield CSRBatch(np.asarray(y, np.float32).reshape(-1, 1), rp, ids, vals)
                k += 1

    def GetTestSamplesSampled(self, sampling_rate: float = 1.0, sampling_max_num: int = 1000000) -> CSRBatch:  # noqa: N802
        if self.mode == "all":
            n = len(self.test)
            k = min(sampling_max_num, int(sampling_rate * n))
            rows = self.rng.choice(n, size=k, replace=False) if k else np.zeros(0, np.int64)
            return self.test.take(np.sort(rows))
        parts = []
        for b in self.NextBatch("test", max_batches=max(1, sampling_max_num // self.batch_size)):
            parts.append(CSRData(b.labels, b.offsets, b.ids, b.vals))
        d = CSRData.concat(parts)
        return d.slice(0, len(d))


def write_synthetic(path_prefix: str, num_files: int, rows_per_file: int, num_features: int,
                    nnz_per_row: int = 20, seed: int = 0, zipf_a: float = 1.2) -> List[str]:
    """Synthetic libsvm shards with a planted linear model (power-law ids) --
    the stand-in for the reference's HDFS click logs (no dataset access)."""
    rng = np.random.default_rng(seed)
    w_true = rng.standard_normal(min(num_features, 1 << 22)).astype(np.float32)
    files = []
    os.makedirs(os.path.dirname(os.path.abspath(path_prefix)) or ".", exist_ok=True)
    for f in range(num_files):
        nnz = rng.integers(max(1, nnz_per_row // 2), nnz_per_row * 3 // 2 + 1, rows_per_file)
        ids = (rng.zipf(zipf_a, int(nnz.sum())) - 1) % num_features
        vals = np.round(rng.random(len(ids)) + 0.5, 3).astype(np.float32)
        offs = np.concatenate([[0], np.cumsum(nnz)])
        logit = np.add.reduceat(w_true[ids % len(w_true)] * vals, offs[:-1]) * 0.5
        y = (rng.random(rows_per_file) < 1 / (1 + np.exp(-logit))).astype(int)
        p = f"{path_prefix}-{f:05d}"
        with open(p, "w") as fh:
            for r in range(rows_per_file):
                s, e = offs[r], offs[r + 1]
                fh.write(f"{y[r]} " + " ".join(f"{i}:{v:g}" for i, v in zip(ids[s:e], vals[s:e])) + "\n")
        files.append(p)
    return files
