"""Asynchronous (Hogwild) parameter-server mode -- the reference's default update
rule (example.py:106-118 without SyncReplicasOptimizer): parallel/async_ps.py,
compat Optimizer(update_mode="async"), examples/mnist_example.py --update_mode=async."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_update_mode_selection(monkeypatch):
    from distributed_tensorflow_example_amd.parallel import async_ps

    monkeypatch.delenv("DTF_UPDATE_MODE", raising=False)
    assert async_ps.update_mode() == "sync"
    monkeypatch.setenv("DTF_UPDATE_MODE", "async")
    assert async_ps.update_mode() == "async"
    assert async_ps.update_mode("sync") == "sync"
    with pytest.raises(ValueError):
        async_ps.update_mode("hogwild")


def test_local_store_is_plain_sgd():
    from distributed_tensorflow_example_amd.parallel import async_ps

    w = torch.arange(6.0).view(2, 3)
    b = torch.ones(4)
    st = async_ps.HogwildStore([w, b], None)
    assert st.kind == "local"
    g = st.sgd_step([torch.ones(2, 3), torch.full((4,), 2.0)], 0.5)
    assert g == 1 and st.global_step() == 1
    assert torch.equal(w, torch.arange(6.0).view(2, 3) - 0.5)
    assert torch.equal(b, torch.zeros(4))


def _shm_worker(rank, ws, port, q, steps, locking):
    try:
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(ws), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(port))
        sys.path.insert(0, REPO)
        from distributed_tensorflow_example_amd.parallel import async_ps
        from distributed_tensorflow_example_amd.parallel import world as W

        w = W.init(backend="gloo")
        p = torch.full((1000,), 100.0) if rank == 0 else torch.zeros(1000)   # the chief's values win
        st = async_ps.HogwildStore([p], w, use_locking=locking)
        assert st.kind == "shm"
        assert torch.equal(p, torch.full((1000,), 100.0)) or rank != 0
        st.pull()
        assert torch.equal(p, torch.full((1000,), 100.0))
        w.barrier()          # (test only: nobody updates before every rank checked the initial values)
        gsteps = []
        for _ in range(steps):
            # integer-valued updates: the locked sum is exact in any order
            gsteps.append(st.sgd_step([torch.full((1000,), float(rank + 1))], 1.0))
        w.barrier()
        st.pull()
        q.put((rank, "ok", p.tolist()[:3], st.global_step(), gsteps))
        w.barrier()
        st.close()
    except Exception:
        import traceback

        q.put((rank, traceback.format_exc(), None, None, None))


@pytest.mark.parametrize("locking", [True, False])
def test_shm_store_two_workers_gloo(locking):
    ws, steps = 2, 25
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shm_worker, args=(r, ws, port, q, steps, locking)) for r in range(ws)]
    [p.start() for p in procs]
    res = sorted([q.get(timeout=240) for _ in range(ws)], key=lambda r: r[0])
    [p.join(60) for p in procs]
    assert all(r[1] == "ok" for r in res), "\n".join(r[1][-1200:] for r in res)
    # every worker's step counted once: global steps 1..50 handed out without duplicates
    allg = sorted(res[0][4] + res[1][4])
    assert allg == list(range(1, ws * steps + 1))
    assert res[0][3] == res[1][3] == ws * steps
    if locking:   # no lost update: 100 - 25 * (1 + 2)
        assert res[0][2] == res[1][2] == [25.0] * 3
    else:         # Hogwild may lose concurrent updates, never invent any
        assert all(25.0 <= v <= 75.0 for v in res[0][2])


def test_mnist_example_async_ps_two_workers(tmp_path):
    """examples/mnist_example.py --update_mode=async as 1 ps + 2 workers on CPU:
    global_step counts both workers' updates, workers finish independently."""
    ports = [_free_port() for _ in range(3)]
    common = [f"--ps_hosts=127.0.0.1:{ports[0]}", f"--worker_hosts=127.0.0.1:{ports[1]},127.0.0.1:{ports[2]}",
              "--max_steps=60", "--train_size=3000", "--frequency=20", f"--logs_path={tmp_path}/logs",
              "--learning_rate=0.05", "--update_mode=async"]
    env = dict(os.environ, PYTHONPATH=REPO, DTF_RENDEZVOUS_TIMEOUT="120")
    script = os.path.join(REPO, "examples", "mnist_example.py")
    procs = {"ps": subprocess.Popen([sys.executable, script, "--job_name=ps", "--task_index=0"] + common, env=env,
                                    stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)}
    for i in (1, 0):
        procs[f"w{i}"] = subprocess.Popen(
            [sys.executable, script, "--job_name=worker", f"--task_index={i}", f"--result_json={tmp_path}/w{i}.json"]
            + common, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    outs = {}
    try:
        for k, pr in procs.items():
            outs[k] = pr.communicate(timeout=240)[0]
    finally:
        for pr in procs.values():
            if pr.poll() is None:
                pr.kill()
    for k, pr in procs.items():
        assert pr.returncode == 0, f"{k} failed:\n{outs.get(k)}"
    r0 = json.load(open(tmp_path / "w0.json"))
    r1 = json.load(open(tmp_path / "w1.json"))
    # each worker stops once the SHARED step reached 60: about 60 updates in all, ~30 each
    assert 60 <= max(r0["global_step"], r1["global_step"]) <= 62, (r0["global_step"], r1["global_step"])
    assert "Test-Accuracy:" in outs["w0"] and "ps 0 done" in outs["ps"]
    assert r0["cost"] == r0["cost"] and r1["cost"] == r1["cost"]   # finite
