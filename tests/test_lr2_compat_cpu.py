"""lr2.py as written through the compat API (examples/lr2_compat.py) on a
ps + 2-worker gloo cluster: the Session's lowered sparse-LR train run
(compat/lowering.py SparseLRStepPlan) trains exactly like the native
SparseLRTrainer program (examples/sparse_lr.py) and like the same graph run
op by op (DTF_GRAPH_LOWERING=0)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def svm(tmp_path_factory):
    sys.path.insert(0, REPO)
    from distributed_tensorflow_example_amd.data import libsvm

    d = tmp_path_factory.mktemp("lr2c")
    tr = libsvm.write_synthetic(str(d / "train" / "part"), 4, 500, 3000, 12, seed=0)
    te = libsvm.write_synthetic(str(d / "test" / "part"), 2, 300, 3000, 12, seed=1)
    return d, tr, te


def _cluster(tmp_path, script, extra, env_extra=None):
    conf = tmp_path / "cluster_conf.json"
    conf.write_text(json.dumps({"ps": [f"127.0.0.1:{_free_port()}"],
                                "worker": [f"127.0.0.1:{_free_port()}", f"127.0.0.1:{_free_port()}"]}))
    env = dict(os.environ, PYTHONPATH=REPO, DTF_RENDEZVOUS_TIMEOUT="120", DTF_SHARD_MIN_ROWS="1000",
               **(env_extra or {}))
    common = [f"--cluster_conf={conf}"] + extra
    path = os.path.join(REPO, "examples", script)
    procs = [subprocess.Popen([sys.executable, path, "--job_name=ps", "--task_index=0"] + common, env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)]
    for i in (1, 0):
        procs.append(subprocess.Popen([sys.executable, path, "--job_name=worker", f"--task_index={i}",
                                       f"--result_json={tmp_path}/w{i}.json"] + common, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for pr in procs:
            outs.append(pr.communicate(timeout=240)[0])
    finally:
        for pr in procs:
            if pr.poll() is None:
                pr.kill()
    for pr, o in zip(procs, outs):
        assert pr.returncode == 0, o[-3000:]
    return [json.load(open(tmp_path / f"w{i}.json")) for i in (0, 1)], outs


def test_lr2_compat_lowered_matches_native_and_op_by_op(svm, tmp_path):
    from distributed_tensorflow_example_amd.compat import saver

    d, tr, te = svm
    common = [f"--train={','.join(tr)}", f"--test={','.join(te)}", "--features=3000", "--num_epochs=2",
              "--learning_rate=0.5", "--batch_size=100", "--trace_step_interval=4"]
    (tmp_path / "low").mkdir()
    (tmp_path / "eager").mkdir()
    (tmp_path / "native").mkdir()
    low, outs = _cluster(tmp_path / "low", "lr2_compat.py", common)
    eager, _ = _cluster(tmp_path / "eager", "lr2_compat.py", common, {"DTF_GRAPH_LOWERING": "0"})
    native, _ = _cluster(tmp_path / "native", "sparse_lr.py",
                         common + ["--seed=0", f"--checkpoint={tmp_path}/native/ck/lr"])
    steps = 2 * 10                                      # 2 epochs x (1000 samples per worker / 100)
    for r in low + eager:
        assert r["steps"] == steps and r["global_step"] == steps
    assert low[0]["lowered_steps"] == steps and eager[0]["lowered_steps"] == 0
    assert "Finish evaluate, auc:" in outs[2]
    w_low = np.load(str(tmp_path / "low" / "w0.json") + ".W.npy")
    w_eager = np.load(str(tmp_path / "eager" / "w0.json") + ".W.npy")
    w_low1 = np.load(str(tmp_path / "low" / "w1.json") + ".W.npy")
    assert np.array_equal(w_low, w_low1)                          # replicas agree
    assert np.allclose(w_low, w_eager, atol=1e-5), np.abs(w_low - w_eager).max()
    assert abs(low[0]["b"] - eager[0]["b"]) < 1e-5
    ck = [p for p in os.listdir(tmp_path / "native" / "ck") if p.endswith(".index")]
    w_nat = saver.read_tensor(str(tmp_path / "native" / "ck" / ck[0][:-6]), "weights/Variable").numpy().reshape(-1)
    assert np.allclose(w_low, w_nat, atol=1e-5), np.abs(w_low - w_nat).max()
    assert abs(low[0]["b"] - native[0]["b"]) < 1e-5
    assert abs(low[0]["loss"] - eager[0]["loss"]) < 1e-4


def test_lr2_compat_one_worker_non_canonical_coo_still_lowers(svm, tmp_path):
    """Worker 1 feeds its COO entries in reverse order: the lower / fall-back
    decision must not differ between ranks (mismatched collectives would hang),
    so that worker's batch is re-sorted by row and both workers lower; the
    result equals the canonical-order run."""
    d, tr, te = svm
    common = [f"--train={','.join(tr)}", f"--test={','.join(te)}", "--features=3000", "--num_epochs=1",
              "--learning_rate=0.5", "--batch_size=100", "--trace_step_interval=4"]
    (tmp_path / "canon").mkdir()
    (tmp_path / "perm").mkdir()
    canon, _ = _cluster(tmp_path / "canon", "lr2_compat.py", common)
    perm, _ = _cluster(tmp_path / "perm", "lr2_compat.py", common, {"DTF_LR2_PERMUTE_COO_TASK": "1"})
    for r in perm:
        assert r["lowered_steps"] == 10 and r["global_step"] == 10
    w_c = np.load(str(tmp_path / "canon" / "w0.json") + ".W.npy")
    w_p = np.load(str(tmp_path / "perm" / "w0.json") + ".W.npy")
    assert np.array_equal(w_p, np.load(str(tmp_path / "perm" / "w1.json") + ".W.npy"))
    assert np.allclose(w_c, w_p, atol=1e-6), np.abs(w_c - w_p).max()


def test_lr2_compat_tensor_feeds_go_op_by_op_on_every_worker(svm, tmp_path):
    """Both workers feed torch tensors: the lowered step takes numpy feeds only,
    and since feed kinds are rank-independent every worker runs op by op (no
    raise, no desynchronised collectives); the result equals the lowered run."""
    d, tr, te = svm
    common = [f"--train={','.join(tr)}", f"--test={','.join(te)}", "--features=3000", "--num_epochs=1",
              "--learning_rate=0.5", "--batch_size=100", "--trace_step_interval=4"]
    (tmp_path / "canon").mkdir()
    (tmp_path / "tens").mkdir()
    canon, _ = _cluster(tmp_path / "canon", "lr2_compat.py", common)
    tens, _ = _cluster(tmp_path / "tens", "lr2_compat.py", common, {"DTF_LR2_TENSOR_FEEDS": "1"})
    for r in tens:
        assert r["lowered_steps"] == 0 and r["global_step"] == 10
    w_c = np.load(str(tmp_path / "canon" / "w0.json") + ".W.npy")
    w_t = np.load(str(tmp_path / "tens" / "w0.json") + ".W.npy")
    assert np.array_equal(w_t, np.load(str(tmp_path / "tens" / "w1.json") + ".W.npy"))
    assert np.allclose(w_c, w_t, atol=1e-5), np.abs(w_c - w_t).max()
