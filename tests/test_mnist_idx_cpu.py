"""Real-MNIST ingestion (the reference's `input_data.read_data_sets(path,
one_hot=True)`, example.py:60-62): IDX files parsed when present, plain or
gzip, TF's 55k/5k train/validation split, synthetic fallback otherwise.  The
fixtures are generated here (no network, no real MNIST in the image); the
header bytes are checked against the IDX spec byte for byte."""
import gzip
import json
import os
import struct
import subprocess
import sys

import numpy as np
import pytest

from distributed_tensorflow_example_amd.data import mnist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _fixture(d, n_train, n_test, gz, seed=0):
    rng = np.random.default_rng(seed)
    xi = rng.integers(0, 256, (n_train, 784), dtype=np.uint8)
    yi = rng.integers(0, 10, n_train, dtype=np.uint8)
    xt = rng.integers(0, 256, (n_test, 784), dtype=np.uint8)
    yt = rng.integers(0, 10, n_test, dtype=np.uint8)
    sfx = ".gz" if gz else ""
    mnist.write_idx_images(os.path.join(d, mnist.TRAIN_IMAGES + sfx), xi)
    mnist.write_idx_labels(os.path.join(d, mnist.TRAIN_LABELS + sfx), yi)
    mnist.write_idx_images(os.path.join(d, mnist.TEST_IMAGES + sfx), xt)
    mnist.write_idx_labels(os.path.join(d, mnist.TEST_LABELS + sfx), yt)
    return xi, yi, xt, yt


def test_idx_header_bytes_exact(tmp_path):
    x = np.arange(3 * 784, dtype=np.uint32).astype(np.uint8).reshape(3, 784)
    p = str(tmp_path / "imgs")
    mnist.write_idx_images(p, x)
    raw = open(p, "rb").read()
    # magic 0x00000803, count 3, rows 28, cols 28 -- all big-endian
    assert raw[:16] == bytes([0, 0, 8, 3, 0, 0, 0, 3, 0, 0, 0, 28, 0, 0, 0, 28])
    assert raw[16:] == x.tobytes() and len(raw) == 16 + 3 * 784
    q = str(tmp_path / "labs")
    mnist.write_idx_labels(q, np.array([7, 2, 1], np.uint8))
    assert open(q, "rb").read() == bytes([0, 0, 8, 1, 0, 0, 0, 3, 7, 2, 1])
    assert np.array_equal(mnist.read_idx_images(p), x)
    assert np.array_equal(mnist.read_idx_labels(q), [7, 2, 1])


@pytest.mark.parametrize("gz", [False, True])
def test_read_data_sets_parses_idx_with_tf_split(tmp_path, gz):
    xi, yi, xt, yt = _fixture(str(tmp_path), 600, 100, gz)
    ds = mnist.read_data_sets(str(tmp_path), one_hot=True, validation_size=50)
    assert ds.source.startswith("idx:")
    assert ds.validation.num_examples == 50 and ds.train.num_examples == 550 and ds.test.num_examples == 100
    assert np.array_equal(ds.validation.images_u8, xi[:50])
    assert np.array_equal(ds.train.images_u8, xi[50:])
    assert np.array_equal(ds.train.labels_u8, yi[50:])
    assert np.array_equal(ds.test.images_u8, xt) and np.array_equal(ds.test.labels_u8, yt)
    # as example.py feeds them: float32 in [0, 1] and one-hot labels
    assert ds.test.images.dtype == np.float32 and np.allclose(ds.test.images, xt / 255.0)
    assert np.array_equal(ds.test.labels.argmax(1), yt) and ds.test.labels.shape == (100, 10)
    bx, by = ds.train.next_batch(100)
    assert bx.shape == (100, 784) and by.shape == (100, 10)


def test_gz_file_is_really_gzip(tmp_path):
    _fixture(str(tmp_path), 10, 10, gz=True)
    with open(tmp_path / (mnist.TRAIN_IMAGES + ".gz"), "rb") as f:
        assert f.read(2) == b"\x1f\x8b"
    with gzip.open(tmp_path / (mnist.TRAIN_LABELS + ".gz")) as f:
        assert struct.unpack(">II", f.read(8)) == (2049, 10)


def test_default_validation_size_is_5000(tmp_path):
    _fixture(str(tmp_path), 6000, 20, gz=True)
    ds = mnist.read_data_sets(str(tmp_path))
    assert ds.validation.num_examples == 5000 and ds.train.num_examples == 1000


def test_bad_magic_and_truncation_raise(tmp_path):
    p = tmp_path / "bad"
    p.write_bytes(struct.pack(">IIII", 2049, 1, 28, 28) + bytes(784))
    with pytest.raises(ValueError, match="magic"):
        mnist.read_idx_images(str(p))
    p.write_bytes(struct.pack(">IIII", 2051, 2, 28, 28) + bytes(784))
    with pytest.raises(ValueError, match="expected"):
        mnist.read_idx_images(str(p))


def test_missing_files_fall_back_to_synthetic(tmp_path):
    ds = mnist.read_data_sets(str(tmp_path / "nothing"), train_size=300, test_size=50, validation_size=20)
    assert ds.source == "synthetic"
    assert (ds.train.num_examples, ds.validation.num_examples, ds.test.num_examples) == (300, 20, 50)
    with pytest.raises(FileNotFoundError):
        mnist.read_data_sets(str(tmp_path / "nothing"), synthetic_fallback=False)


def test_mnist_example_trains_on_idx_dir(tmp_path):
    """examples/mnist_example.py (single worker, CPU) reads the IDX directory
    given by --data_dir and its Test-Accuracy is computed on the t10k split."""
    d = tmp_path / "mnist"
    d.mkdir()
    # a learnable fixture: the synthetic prototypes, written as IDX files
    xi, yi = mnist.synthetic_mnist(6000, seed=3)   # 5000 validation + 1000 train
    xt, yt = mnist.synthetic_mnist(200, seed=4)
    mnist.write_idx_images(str(d / (mnist.TRAIN_IMAGES + ".gz")), xi)
    mnist.write_idx_labels(str(d / (mnist.TRAIN_LABELS + ".gz")), yi)
    mnist.write_idx_images(str(d / mnist.TEST_IMAGES), xt)
    mnist.write_idx_labels(str(d / mnist.TEST_LABELS), yt)
    res = tmp_path / "res.json"
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, os.path.join(REPO, "examples", "mnist_example.py"), "--job_name=worker", "--task_index=0",
           "--ps_hosts=", f"--worker_hosts=127.0.0.1:{port}", f"--data_dir={d}", "--training_epochs=10",
           "--learning_rate=0.5", f"--logs_path={tmp_path / 'logs'}", f"--result_json={res}"]
    env = dict(os.environ, PYTHONPATH=REPO, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert f"MNIST source: idx:{d}" in r.stdout
    assert "train 1000, validation 5000, test 200" in r.stdout   # TF's split of the training file
    out = json.loads(res.read_text())
    assert out["accuracy"] > 0.3, out   # well above chance (0.1) on the t10k fixture
