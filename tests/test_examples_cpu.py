"""The reference's side programs, run end to end on CPU: model_export.py,
the two input-pipeline demos, hdfs_test.py (fake HDFS), and the launcher
(file lists, local cluster, failure teardown)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, PYTHONPATH=REPO)


def _run(args, timeout=240, env=None):
    p = subprocess.run([sys.executable] + args, capture_output=True, text=True, timeout=timeout, env=env or ENV,
                       cwd=REPO)
    return p.returncode, p.stdout + p.stderr


def test_model_export(tmp_path):
    rc, out = _run(["examples/model_export.py", f"--work_dir={tmp_path}/model", "--n_steps=500"])
    assert rc == 0, out
    d = tmp_path / "model" / "00000003"
    assert (d / "export.index").exists() and (d / "export.data-00000-of-00001").exists()
    assert (d / "export.meta").exists() and (d / "checkpoint").exists()
    sys.path.insert(0, REPO)
    from distributed_tensorflow_example_amd.compat import export
    from distributed_tensorflow_example_amd.compat import meta_graph as M

    meta = M.parse_meta_graph((d / "export.meta").read_bytes())
    sigs = M.parse_signatures(meta["collection_def"]["serving_signatures"]["value"][0]["value"])["named_signatures"]
    assert set(sigs) == {"inputs", "outputs"}
    assert sigs["inputs"] == {"kind": "generic", "map": {"x": "x:0"}}
    assert sigs["outputs"]["map"]["y"] == "test/add:0"
    names = [M.parse_variable_def(v)["variable_name"] for v in meta["collection_def"]["variables"]["value"]]
    assert {"test/weights:0", "test/bias:0", "test/weights/Adam:0", "beta1_power:0"} <= set(names)
    # y = x + 20 sin(x/10) on [0, 100): least squares slope ~ 0.97 -- 500 Adam steps get close
    b = export.load_session_bundle(str(d))
    w = float(b.tensors["test/weights"].reshape(-1)[0])
    assert 0.5 < w < 1.5


def test_input_pipeline_demo(tmp_path):
    rc, out = _run(["examples/input_pipeline.py", f"--dataset_path={tmp_path}/ds/", "--train_batches=6",
                    "--test_batches=4"])
    assert rc == 0, out
    assert "from the train set:" in out and "from the test set:" in out


def test_input_pipeline_large_dataset_demo():
    rc, out = _run(["examples/input_pipeline_large_dataset.py", "--batches=7000"])   # wraps past 100,003 rows
    assert rc == 0, out
    assert "dequeued 7000 batches" in out


def test_hdfs_line_count_threads(tmp_path):
    root = tmp_path / "hdfs"
    (root / "d").mkdir(parents=True)
    for i, n in enumerate((10, 20, 30)):
        (root / "d" / f"part-{i:05d}").write_text("x\n" * n)
    files = ",".join(f"hdfs://localhost:9000/d/part-{i:05d}" for i in range(3))
    rc, out = _run(["examples/hdfs_test.py", f"--files={files}"], env=dict(ENV, DTF_FAKE_HDFS_ROOT=str(root)))
    assert rc == 0, out
    for i, n in enumerate((10, 20, 30)):
        assert f"thread: {i}, lines: {n}," in out


def test_launcher_filelist_and_failure_teardown(tmp_path):
    d = tmp_path / "data"
    d.mkdir()
    (d / "small").write_text("1 1:1\n")
    (d / "sub").mkdir()
    (d / "sub" / "big").write_text("1 1:1\n" * 400)
    (d / "big2").write_text("0 2:1\n" * 400)
    rc, out = _run(["-m", "distributed_tensorflow_example_amd.launch", "filelist", str(d), "-R", "--min-size",
                    "1000"])
    assert rc == 0
    assert out.strip() == f"{d}/big2,{d}/sub/big"
    # a worker that dies must take the ps (blocked in join) down with it
    bad = tmp_path / "bad.py"
    bad.write_text(
        "import sys, json\n"
        f"sys.path.insert(0, {REPO!r})\n"
        "import distributed_tensorflow_example_amd.compat as tf\n"
        "tf.app.flags.DEFINE_string('job_name', '', '')\n"
        "tf.app.flags.DEFINE_integer('task_index', 0, '')\n"
        "tf.app.flags.DEFINE_string('cluster_conf', '', '')\n"
        "F = tf.app.flags.FLAGS\n"
        "def main(_):\n"
        "    s = tf.train.Server(tf.train.ClusterSpec(json.load(open(F.cluster_conf))), F.job_name, F.task_index)\n"
        "    if F.job_name == 'ps':\n"
        "        s.join()\n"
        "        return 0\n"
        "    raise SystemExit(3)\n"
        "tf.app.run(main)\n")
    rc, out = _run(["-m", "distributed_tensorflow_example_amd.launch", "local", "--ps", "1", "--workers", "1",
                    "--log-dir", str(tmp_path / "logs"), str(bad)], timeout=120)
    assert rc == 3, out
    assert "failed" in out and "stopping the job" in out
