"""The reference's own program (examples/mnist_example.py = example.py's graph
under replica_device_setter + Supervisor + sess.run) as synchronous data
parallelism with 1 ps + 2 and 1 ps + 4 workers sharing cuda:0: every
Session.run of the train op is the lowered native step whose last kernel
all-reduces the workers' gradients over the IPC data plane and applies SGD
(csrc/bind_mlp.cpp GraphStepPlan.attach_ipc, csrc/kernels/ipc_coll.hip
reduce_sgd_k).  No RCCL communicator is created; the replicas are
bit-identical; the parameters after 20 steps match an fp64 evaluation of
example.py's graph trained on the worker-averaged gradient (1e-5 relative).
Reference: example.py:64-67,109-123,139-171; README.md:11-16."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_cluster(tmp, workers, steps, extra=(), env_extra=None, timeout=400):
    conf = os.path.join(tmp, "cluster.json")
    with open(conf, "w") as f:
        json.dump({"ps": [f"127.0.0.1:{_port()}"], "worker": [f"127.0.0.1:{_port()}" for _ in range(workers)]}, f)
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="2", DTF_RENDEZVOUS_TIMEOUT="180",
               DTF_IPC_TIMEOUT_S="60", **(env_extra or {}))
    ex = os.path.join(REPO, "examples", "mnist_example.py")
    common = [f"--cluster_conf={conf}", f"--max_steps={steps}", "--train_size=3000", "--frequency=1000000",
              f"--logs_path={tmp}/logs", f"--dump_dir={tmp}/dump", "--data_dir=/nonexistent"] + list(extra)
    procs = [subprocess.Popen([sys.executable, ex, "--job_name=ps", "--task_index=0"] + common, env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)]
    for i in range(workers):
        procs.append(subprocess.Popen([sys.executable, ex, "--job_name=worker", f"--task_index={i}"] + common,
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=timeout)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-4000:]
    dumps = [dict(np.load(os.path.join(tmp, "dump", f"worker_{i}.npz"))) for i in range(workers)]
    facts = [json.load(open(os.path.join(tmp, "dump", f"worker_{i}.json"))) for i in range(workers)]
    return dumps, facts, outs


def _ref_train(init, batches, lr):
    """fp64 autograd through example.py's literal graph (naive xent), gradient
    averaged over the workers' batches each step."""
    W1, W2, b1, b2 = [torch.tensor(p, dtype=torch.float64) for p in init]
    for per_worker in batches:
        gs = []
        for bx, by in per_worker:
            ps = [t.clone().requires_grad_(True) for t in (W1, W2, b1, b2)]
            x, y_ = torch.tensor(bx, dtype=torch.float64), torch.tensor(by, dtype=torch.float64)
            y = torch.softmax(torch.sigmoid(x @ ps[0] + ps[2]) @ ps[1] + ps[3], 1)
            ce = (-(y_ * torch.log(y)).sum(1)).mean()
            ce.backward()
            gs.append([p.grad for p in ps])
        W1, W2, b1, b2 = [p - lr * sum(g[k] for g in gs) / len(gs) for k, p in enumerate((W1, W2, b1, b2))]
    return [t.numpy() for t in (W1, W2, b1, b2)]


@pytest.mark.parametrize("workers", [2, 4])
def test_mnist_example_sync_workers_on_ipc_plane(tmp_path, workers):
    steps, lr = 20, 0.05
    dumps, facts, _ = run_cluster(str(tmp_path), workers, steps, extra=[f"--learning_rate={lr}"])
    for f in facts:
        assert f["world_size"] == workers and f["steps"] == steps
        assert f["native_plan_ipc"] and f["native_plan_steps"] == steps, f
        assert not f["rccl_comm"], f               # no RCCL communicator anywhere
        assert f["ipc_calls"] >= steps, f
    # chief init + broadcast: every worker started from the same parameters
    for d in dumps[1:]:
        for k in range(4):
            assert np.array_equal(d[f"init{k}"], dumps[0][f"init{k}"])
    # bit-identical replicas
    for d in dumps[1:]:
        for k in range(4):
            assert np.array_equal(d[f"final{k}"], dumps[0][f"final{k}"]), k
    init = [dumps[0][f"init{k}"] for k in range(4)]
    batches = [[(d["xs"][s], d["ys"][s]) for d in dumps] for s in range(steps)]
    ref = _ref_train(init, batches, lr)
    for k in range(4):
        got = dumps[0][f"final{k}"]
        rel = np.abs(got - ref[k]).max() / max(np.abs(ref[k]).max(), 1e-30)
        assert rel <= 1e-5, (k, rel)
        # and the training itself (the parameter change), not only the values
        dg, dr = got.astype(np.float64) - init[k], ref[k] - init[k]
        assert np.abs(dr).max() > 0
        assert np.abs(dg - dr).max() <= 1e-3 * np.abs(dr).max(), k
