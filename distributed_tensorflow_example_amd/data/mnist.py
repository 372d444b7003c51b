"""Synthetic MNIST-shaped data (no network: the reference downloads MNIST via
`input_data.read_data_sets`, example.py:59-62; we generate data of the same
shape/dtype instead).

Images are uint8 [N, 784] (the IDX file's native pixel format), labels uint8
class ids [N].  Each class has a random low-frequency prototype; samples are
prototype + noise, so a 784-100-10 MLP learns it and accuracy is meaningful.

`PinnedEpoch` packs a whole epoch batch-major into pinned host memory:
record b = [B*784 pixels | B labels | pad to 16 B], which is what the input
pipeline streams to the GPU with one hipMemcpyAsync per step on a side stream.
"""
from __future__ import annotations

import numpy as np
import torch

IMAGE_PIXELS = 784
NUM_CLASSES = 10
TRAIN_EXAMPLES = 55000  # mnist.train.num_examples used by example.py:161
TEST_EXAMPLES = 10000


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
    float images in [0,1] and one-hot labels as the reference feeds them)."""

    def __init__(self, images_u8: np.ndarray, labels_u8: np.ndarray, seed: int = 0, shuffle: bool = True):
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
        return self.images_u8[idx].astype(np.float32) / 255.0, one_hot(self.labels_u8[idx])


class Datasets:
    def __init__(self, train: DataSet, test: DataSet):
        self.train = train
        self.test = test


def read_data_sets(train_dir: str = "", one_hot: bool = True, seed: int = 0,
                   train_size: int = TRAIN_EXAMPLES, test_size: int = TEST_EXAMPLES) -> Datasets:
    """Synthetic drop-in for tensorflow.examples.tutorials.mnist.input_data.read_data_sets."""
    del train_dir, one_hot
    xi, yi = synthetic_mnist(train_size, seed=seed)
    xt, yt = synthetic_mnist(test_size, seed=seed + 7919)
    return Datasets(DataSet(xi, yi, seed=seed), DataSet(xt, yt, seed=seed, shuffle=False))


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
