"""Failure detection + checkpoint restart: a worker
killed by fault injection tears the whole ps/worker job down through the
launcher; restarting the job resumes from the chief's last checkpoint and
finishes at the requested global step.  Also: replica-consistency checks and
the profiling / metrics utilities."""
import json
import os
import subprocess
import sys

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launch(tmp_path, extra_env, logs, max_steps=60):
    env = dict(os.environ, PYTHONPATH=REPO, DTF_RENDEZVOUS_TIMEOUT="60", DTF_PEER_TIMEOUT="5", **extra_env)
    cmd = [sys.executable, "-m", "distributed_tensorflow_example_amd.launch", "local", "--ps", "1", "--workers", "2",
           "--log-dir", str(tmp_path / logs), "--timeout", "200", os.path.join(REPO, "examples", "mnist_example.py"),
           "--", f"--max_steps={max_steps}", "--train_size=3000", "--frequency=10",
           f"--logs_path={tmp_path}/tb", "--learning_rate=0.05", f"--checkpoint_dir={tmp_path}/ckpt",
           "--save_model_steps=10", f"--metrics_jsonl={tmp_path}/m_{logs}.jsonl",
           f"--result_json={tmp_path}/r_{logs}.json"]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))


def test_worker_fault_teardown_and_checkpoint_restart(tmp_path):
    r1 = _launch(tmp_path, {"DTF_FAULT_STEP": "25", "DTF_FAULT_RANK": "1"}, "run1")
    assert r1.returncode != 0, r1.stdout + r1.stderr
    assert "failed" in r1.stdout and "stopping the job" in r1.stdout
    w1 = open(tmp_path / "run1" / "worker_1.log").read()
    assert "injected fault at step 25" in w1
    sys.path.insert(0, REPO)
    import distributed_tensorflow_example_amd.compat as tf

    ck = tf.train.latest_checkpoint(str(tmp_path / "ckpt"))
    assert ck is not None and ck.endswith("-20"), ck
    r2 = _launch(tmp_path, {}, "run2")
    assert r2.returncode == 0, r2.stdout + r2.stderr + open(tmp_path / "run2" / "worker_0.log").read()
    w0 = open(tmp_path / "run2" / "worker_0.log").read()
    assert "restored from checkpoint at global step 20" in w0
    res = json.load(open(tmp_path / "r_run2.json"))
    assert res["global_step"] == 60
    steps = [json.loads(l)["step"] for l in open(tmp_path / "m_run2.jsonl") if '"kind": "step"' in l]
    assert min(steps) == 21 and max(steps) == 60
    assert tf.train.latest_checkpoint(str(tmp_path / "ckpt")).endswith("-60")


def test_replica_checksum_detects_divergence():
    sys.path.insert(0, REPO)
    from distributed_tensorflow_example_amd.utils import debug

    a = [torch.arange(10.0), torch.ones(3)]
    b = [torch.arange(10.0).flip(0), torch.ones(3)]          # same sum, different order
    assert not torch.equal(debug.replica_checksum(a), debug.replica_checksum(b))

    class FakeWorld:
        world_size = 1
    assert debug.assert_replicas_consistent(FakeWorld(), a)
    os.environ["DTF_FAULT_STEP"] = "3"
    os.environ["DTF_FAULT_RANK"] = "0"
    try:
        debug.fault_point(2, 0)
        with pytest.raises(debug.InjectedFault):
            debug.fault_point(3, 0)
        debug.fault_point(3, 1)
    finally:
        del os.environ["DTF_FAULT_STEP"], os.environ["DTF_FAULT_RANK"]


def test_profiling_and_metrics(tmp_path):
    sys.path.insert(0, REPO)
    from distributed_tensorflow_example_amd.utils import metrics, profiling

    with profiling.TraceRecorder(str(tmp_path / "trace.json")):
        with profiling.range("fwd"):
            sum(range(1000))
        with profiling.range("bwd"):
            pass
    tr = json.load(open(tmp_path / "trace.json"))
    assert [e["name"] for e in tr["traceEvents"]] == ["fwd", "bwd"]
    t = profiling.StepTimer()
    for _ in range(5):
        t.start()
        t.stop()
    s = t.summary()
    assert s["steps"] == 5 and s["p50_ms"] >= 0 and s["p90_ms"] >= s["p50_ms"]
    with metrics.MetricsWriter(str(tmp_path / "m.jsonl"), rank=3) as mw:
        mw.write("step", 1, loss=torch.tensor(0.5))
    rec = metrics.read_jsonl(str(tmp_path / "m.jsonl"))
    assert rec[0]["rank"] == 3 and rec[0]["loss"] == 0.5 and rec[0]["step"] == 1
