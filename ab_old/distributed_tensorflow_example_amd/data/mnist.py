"""MNIST input: the real IDX files when they are present, synthetic MNIST-shaped
data otherwise.

The reference calls `input_data.read_data_sets(path, one_hot=True)`
(example.py:59-62), which downloads the four IDX files into `path` and splits
the 60,000 training images into `train` (55,000) and `validation` (the first
5,000), with `test` = the 10,000 t10k images (example.py:161,165,187 use
`mnist.train.num_examples`, `mnist.train.next_batch`, `mnist.test.images`).
There is no network here: `read_data_sets` parses the IDX files if they exist
in `train_dir` (plain or `.gz`, TF's file names) and falls back to synthetic
data of the same shape/dtype otherwise, with the same split.

Images are uint8 [N, 784] (the IDX file's native pixel format), labels uint8
class ids [N].  Each class has a random low-frequency prototype; samples are
prototype + noise, so a 784-100-10 MLP learns it and accuracy is meaningful.

`PinnedEpoch` packs a whole epoch batch-major into pinned host memory:
record b = [B*784 pixels | B labels | pad to 16 B], which is what the input
pipeline streams to the GPU with one hipMemcpyAsync per step on a side stream.
"""
from __future__ import annotations

import gzip
import os
import struct
import sys
from typing import Optional

import numpy as np
import torch

IMAGE_PIXELS = 784
NUM_CLASSES = 10
TRAIN_EXAMPLES = 55000  # mnist.train.num_examples used by example.py:161
TEST_EXAMPLES = 10000
VALIDATION_SIZE = 5000  # TF's read_data_sets default split of the 60k training images

TRAIN_IMAGES = "train-images-idx3-ubyte"
TRAIN_LABELS = "train-labels-idx1-ubyte"
TEST_IMAGES = "t10k-images-idx3-ubyte"
TEST_LABELS = "t10k-labels-idx1-ubyte"
IDX_IMAGES_MAGIC = 2051   # 0x00000803: ubyte, 3 dims
IDX_LABELS_MAGIC = 2049   # 0x00000801: ubyte, 1 dim


def _open_idx(path: str):
    return gzip.open(path, "rb") if path.endswith(".gz") else open(path, "rb")


def _find_idx(train_dir: str, name: str):
    """`name` or `name.gz` in train_dir (the plain file wins), else None."""
    for cand in (name, name + ".gz"):
        p = os.path.join(train_dir, cand)
        if os.path.isfile(p):
            return p
    return None


def read_idx_images(path: str) -> np.ndarray:
    """IDX3 ubyte images -> uint8 [N, rows*cols] (big-endian header: magic 2051,
    count, rows, cols; then row-major pixels)."""
    with _open_idx(path) as f:
        head = f.read(16)
        if len(head) != 16:
            raise ValueError(f"{path}: truncated IDX header")
        magic, n, rows, cols = struct.unpack(">IIII", head)
        if magic != IDX_IMAGES_MAGIC:
            raise ValueError(f"{path}: invalid magic number {magic} in MNIST image file")
        data = f.read(n * rows * cols)
    if len(data) != n * rows * cols:
        raise ValueError(f"{path}: expected {n * rows * cols} pixel bytes, got {len(data)}")
    return np.frombuffer(data, dtype=np.uint8).reshape(n, rows * cols).copy()


def read_idx_labels(path: str) -> np.ndarray:
    """IDX1 ubyte labels -> uint8 [N] (magic 2049, count, then one byte per label)."""
    with _open_idx(path) as f:
        head = f.read(8)
        if len(head) != 8:
            raise ValueError(f"{path}: truncated IDX header")
        magic, n = struct.unpack(">II", head)
        if magic != IDX_LABELS_MAGIC:
            raise ValueError(f"{path}: invalid magic number {magic} in MNIST label file")
        data = f.read(n)
    if len(data) != n:
        raise ValueError(f"{path}: expected {n} labels, got {len(data)}")
    return np.frombuffer(data, dtype=np.uint8).copy()


def write_idx_images(path: str, images_u8: np.ndarray, rows: int = 28, cols: int = 28):
    """Write uint8 [N, rows*cols] as an IDX3 file (gzip if path ends in .gz)."""
    images_u8 = np.ascontiguousarray(images_u8, dtype=np.uint8)
    payload = struct.pack(">IIII", IDX_IMAGES_MAGIC, images_u8.shape[0], rows, cols) + images_u8.tobytes()
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "wb") as f:
        f.write(payload)


def write_idx_labels(path: str, labels_u8: np.ndarray):
    labels_u8 = np.ascontiguousarray(labels_u8, dtype=np.uint8)
    payload = struct.pack(">II", IDX_LABELS_MAGIC, labels_u8.shape[0]) + labels_u8.tobytes()
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "wb") as f:
        f.write(payload)


def _prototypes(seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    protos = np.zeros((NUM_CLASSES, 28, 28), np.float32)
    yy, xx = np.mgrid[0:28, 0:28]
    for c in range(NUM_CLASSES):
        for _ in range(3):
            cy, cx = rng.uniform(6, 22, size=2)
            sy, sx = rng.uniform(2.0, 5.0, size=2)
            protos[c] += np.exp(-(((yy - cy) / sy) ** 2 + ((xx - cx) / sx) ** 2))
        protos[c] /= protos[c].max()
    return protos.reshape(NUM_CLASSES, IMAGE_PIXELS)


def synthetic_mnist(n: int, seed: int = 0, proto_seed: int = 1234, noise: float = 0.35):
    """Return (images uint8 [n,784], labels uint8 [n])."""
    rng = np.random.default_rng(seed)
    protos = _prototypes(proto_seed)
    labels = rng.integers(0, NUM_CLASSES, size=n).astype(np.uint8)
    imgs = protos[labels] + noise * rng.standard_normal((n, IMAGE_PIXELS)).astype(np.float32)
    imgs = np.clip(imgs * 255.0, 0, 255).astype(np.uint8)
    return imgs, labels


def one_hot(labels: np.ndarray, n: int = NUM_CLASSES) -> np.ndarray:
    out = np.zeros((labels.shape[0], n), np.float32)
    out[np.arange(labels.shape[0]), labels.astype(np.int64)] = 1.0
    return out


class DataSet:
    """Minimal stand-in for `mnist.train` / `mnist.test` (next_batch, epochs,
    float images in [0,1] and one-hot labels as the reference feeds them).

    `next_batch` returns ordinary writeable float32 arrays, like TF's loader
    (callers may normalise / shuffle / augment a batch in place).  With
    `pixel_batches=True` (opt-in: `read_data_sets(..., pixel_batches=True)` or
    DTF_MNIST_PIXEL_BATCHES=1) it returns read-only `PixelBatch`es instead, which
    the lowered Session step ships as their 4x smaller uint8 source."""

    def __init__(self, images_u8: np.ndarray, labels_u8: np.ndarray, seed: int = 0, shuffle: bool = True,
                 pixel_batches: bool = False):
        self.pixel_batches = bool(pixel_batches)
        self.images_u8 = images_u8
        self.labels_u8 = labels_u8
        self._rng = np.random.default_rng(seed)
        self._shuffle = shuffle
        self._pos = 0
        self.epochs_completed = 0
        self._perm = np.arange(len(labels_u8))

    @property
    def num_examples(self) -> int:
        return len(self.labels_u8)

    @property
    def images(self) -> np.ndarray:
        return self.images_u8.astype(np.float32) / 255.0

    @property
    def labels(self) -> np.ndarray:
        return one_hot(self.labels_u8)

    def next_batch(self, batch_size: int):
        if self._pos + batch_size > self.num_examples:
            self.epochs_completed += 1
            self._pos = 0
            if self._shuffle:
                self._perm = self._rng.permutation(self.num_examples)
        idx = self._perm[self._pos:self._pos + batch_size]
        self._pos += batch_size
        u8 = self.images_u8[idx]
        if self.pixel_batches:
            return PixelBatch.of(u8), one_hot(self.labels_u8[idx])
        return u8.astype(np.float32) / np.float32(255.0), one_hot(self.labels_u8[idx])


class PixelBatch(np.ndarray):
    """A read-only float32 image batch x = u8 / 255 that keeps its uint8 source
    in `.u8` (the loader's opt-in `pixel_batches` mode: read-only, so the source
    provably still matches the floats).  Everywhere it is an ordinary float32 array; the lowered Session
    step (compat/lowering.py) ships the 4x smaller uint8 batch instead and the
    kernel converts with the same correctly rounded float32 division, so the
    step is bit-identical.  Arrays derived from it (slices, arithmetic) carry no
    source."""

    u8 = None

    @staticmethod
    def of(u8: np.ndarray) -> "PixelBatch":
        x = (u8.astype(np.float32) / np.float32(255.0)).view(PixelBatch)
        x.u8 = np.ascontiguousarray(u8)
        x.flags.writeable = False
        return x

    def __array_finalize__(self, obj):
        self.u8 = None

    def __reduce__(self):   # pickles as a plain float32 array
        return np.asarray(self).copy().__reduce__()


class Datasets:
    def __init__(self, train: DataSet, test: DataSet, validation: DataSet = None, source: str = "synthetic"):
        self.train = train
        self.validation = validation
        self.test = test
        self.source = source   # "idx:<dir>" or "synthetic"


def idx_files(train_dir: str):
    """The four IDX paths in train_dir (plain or .gz), or None if any is missing."""
    if not train_dir or not os.path.isdir(train_dir):
        return None
    paths = [_find_idx(train_dir, n) for n in (TRAIN_IMAGES, TRAIN_LABELS, TEST_IMAGES, TEST_LABELS)]
    return None if any(p is None for p in paths) else paths


def read_data_sets(train_dir: str = "", one_hot: bool = True, seed: int = 0,
                   train_size: int = TRAIN_EXAMPLES, test_size: int = TEST_EXAMPLES,
                   validation_size: int = VALIDATION_SIZE, synthetic_fallback: bool = True,
                   pixel_batches: Optional[bool] = None) -> Datasets:
    """Drop-in for tensorflow.examples.tutorials.mnist.input_data.read_data_sets.

    Real data: the IDX files in `train_dir`; the first `validation_size` training
    images become `validation`, the rest `train` (TF's split), `test` = t10k.
    `train_size` / `test_size` only size the synthetic fallback, which has the
    same three splits.  `one_hot` is accepted for signature parity: `labels`
    are always one-hot float32 (what example.py feeds), `labels_u8` the ids.
    `pixel_batches`: next_batch returns read-only `PixelBatch`es (see DataSet);
    None reads DTF_MNIST_PIXEL_BATCHES (default off: writeable float32 batches).
    """
    del one_hot
    if pixel_batches is None:
        pixel_batches = os.environ.get("DTF_MNIST_PIXEL_BATCHES", "0") == "1"
    pb = {"pixel_batches": bool(pixel_batches)}
    paths = idx_files(train_dir)
    if paths is not None:
        xi, yi = read_idx_images(paths[0]), read_idx_labels(paths[1])
        xt, yt = read_idx_images(paths[2]), read_idx_labels(paths[3])
        if len(xi) != len(yi) or len(xt) != len(yt):
            raise ValueError(f"{train_dir}: image / label counts differ ({len(xi)}/{len(yi)}, {len(xt)}/{len(yt)})")
        if not 0 <= validation_size <= len(xi):
            raise ValueError(f"validation size should be between 0 and {len(xi)}; received {validation_size}")
        return Datasets(DataSet(xi[validation_size:], yi[validation_size:], seed=seed, **pb),
                        DataSet(xt, yt, seed=seed, shuffle=False, **pb),
                        DataSet(xi[:validation_size], yi[:validation_size], seed=seed, shuffle=False, **pb),
                        source=f"idx:{os.path.abspath(train_dir)}")
    if not synthetic_fallback:
        raise FileNotFoundError(f"MNIST IDX files not found in {train_dir!r} (no network to download them)")
    if train_dir:
        print(f"read_data_sets: no MNIST IDX files in {train_dir!r}; using synthetic MNIST-shaped data",
              file=sys.stderr, flush=True)
    xi, yi = synthetic_mnist(train_size, seed=seed)
    xv, yv = synthetic_mnist(validation_size, seed=seed + 104729) if validation_size > 0 else (xi[:0], yi[:0])
    xt, yt = synthetic_mnist(test_size, seed=seed + 7919)
    return Datasets(DataSet(xi, yi, seed=seed, **pb), DataSet(xt, yt, seed=seed, shuffle=False, **pb),
                    DataSet(xv, yv, seed=seed, shuffle=False, **pb), source="synthetic")


def record_bytes(batch_size: int) -> int:
    n = batch_size * (IMAGE_PIXELS + 1)
    return (n + 15) // 16 * 16


class PinnedEpoch:
    """A whole epoch packed batch-major in pinned host memory."""

    def __init__(self, images_u8: np.ndarray, labels_u8: np.ndarray, batch_size: int, pin: bool = True):
        n = (len(labels_u8) // batch_size) * batch_size
        self.batch_size = batch_size
        self.num_batches = n // batch_size
        self.rec = record_bytes(batch_size)
        host = torch.zeros((self.num_batches, self.rec), dtype=torch.uint8,
                           pin_memory=pin and torch.cuda.is_available())
        self.host = host
        self._fill(images_u8[:n], labels_u8[:n])

    def _fill(self, images_u8: np.ndarray, labels_u8: np.ndarray):
        B = self.batch_size
        arr = self.host.numpy()
        px = images_u8.reshape(self.num_batches, B * IMAGE_PIXELS)
        lb = labels_u8.reshape(self.num_batches, B)
        arr[:, : B * IMAGE_PIXELS] = px
        arr[:, B * IMAGE_PIXELS: B * IMAGE_PIXELS + B] = lb

    def shuffle(self, seed: int):
        """Re-pack with a new sample permutation (epoch-level shuffle)."""
        B = self.batch_size
        arr = self.host.numpy()
        px = arr[:, : B * IMAGE_PIXELS].reshape(-1, IMAGE_PIXELS).copy()
        lb = arr[:, B * IMAGE_PIXELS: B * IMAGE_PIXELS + B].reshape(-1).copy()
        perm = np.random.default_rng(seed).permutation(len(lb))
        self._fill(px[perm], lb[perm])

    def batch(self, b: int):
        """(images uint8 [B,784], labels uint8 [B]) views of batch b."""
        B = self.batch_size
        rec = self.host[b % self.num_batches]
        return rec[: B * IMAGE_PIXELS].view(B, IMAGE_PIXELS), rec[B * IMAGE_PIXELS: B * IMAGE_PIXELS + B]
