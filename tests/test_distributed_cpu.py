"""Multi-process CPU (gloo) tests of the distributed path: World collectives,
bucketed DDP == single-process large-batch SGD, and the ClusterSpec ps/worker
example (1 ps + 2 workers) training in lock-step (BASELINE config #1 shape)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(rank, ws, port):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(ws), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))


def _collectives_worker(rank, ws, port, q):
    try:
        sys.path.insert(0, REPO)
        _env(rank, ws, port)
        from distributed_tensorflow_example_amd.parallel import world as W

        w = W.init(backend="gloo")
        t = torch.full((5,), float(rank + 1))
        w.all_reduce(t)
        assert torch.allclose(t, torch.full((5,), float(ws * (ws + 1) / 2)))
        b = torch.arange(4.0) if rank == 0 else torch.zeros(4)
        w.broadcast(b, 0)
        assert torch.equal(b, torch.arange(4.0))
        dst = torch.zeros(ws * 3)
        w.all_gather(torch.full((3,), float(rank)), dst)
        assert torch.equal(dst, torch.arange(ws).float().repeat_interleave(3))
        rs = torch.zeros(2)
        w.reduce_scatter(torch.arange(2.0 * ws), rs)
        assert torch.equal(rs, ws * torch.arange(2.0 * rank, 2.0 * rank + 2))
        # all_to_all with uneven splits: rank r sends (j+1) rows to rank j
        send = [j + 1 for j in range(ws)]
        recv = [rank + 1] * ws
        src = torch.cat([torch.full((j + 1,), float(10 * rank + j)) for j in range(ws)])
        out = torch.zeros(sum(recv))
        w.all_to_all(src, send, out, recv)
        exp = torch.cat([torch.full((rank + 1,), float(10 * r + rank)) for r in range(ws)])
        assert torch.equal(out, exp)
        assert w.host_all_reduce(rank, "max") == ws - 1
        assert w.broadcast_object({"r": rank}, 0) == {"r": 0}
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, traceback.format_exc()))


def _ddp_worker(rank, ws, port, q, bucket_mb):
    try:
        sys.path.insert(0, REPO)
        _env(rank, ws, port)
        from distributed_tensorflow_example_amd import optim
        from distributed_tensorflow_example_amd.models.mlp import MLP
        from distributed_tensorflow_example_amd.parallel import world as W
        from distributed_tensorflow_example_amd.parallel.ddp import DistributedDataParallel

        w = W.init(backend="gloo")
        torch.manual_seed(0)
        X = torch.rand(64, 784)
        Y = torch.randint(0, 10, (64,))
        model = MLP(seed=1 + rank)                      # different init: DDP must broadcast rank 0's
        ddp = DistributedDataParallel(model, w, bucket_mb=bucket_mb)
        opt = optim.FusedSGD(list(model.parameters()), 0.1)
        shard = slice(rank * 64 // ws, (rank + 1) * 64 // ws)
        for _ in range(3):
            ddp.zero_grad()
            loss = torch.nn.functional.cross_entropy(ddp(X[shard]), Y[shard])
            loss.backward()
            ddp.finish_gradient_synchronization()
            opt.step()
        q.put((rank, [p.detach().numpy().copy() for p in model.parameters()], len(ddp.buckets)))
    except Exception:
        import traceback

        q.put((rank, traceback.format_exc(), 0))


def _spawn(fn, ws, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=fn, args=(r, ws, port, q) + args) for r in range(ws)]
    [p.start() for p in procs]
    res = [q.get(timeout=240) for _ in range(ws)]
    [p.join(60) for p in procs]
    return sorted(res, key=lambda r: r[0])


@pytest.mark.parametrize("ws", [2, 3, 4, 8])
def test_world_collectives_gloo(ws):
    res = _spawn(_collectives_worker, ws)
    for r in res:
        assert r[1] == "ok", r[1]


@pytest.mark.parametrize("bucket_mb,ws", [(25.0, 2), (0.001, 2), (0.001, 4), (25.0, 8), ("auto", 2), ("measure", 2)])
def test_ddp_matches_full_batch_sgd(bucket_mb, ws):
    res = _spawn(_ddp_worker, ws, bucket_mb)
    for r in res:
        assert isinstance(r[1], list), r[1]
    if not isinstance(bucket_mb, str) and bucket_mb < 1:
        assert res[0][2] > 1                            # really bucketed
    from distributed_tensorflow_example_amd.models.mlp import MLP

    torch.manual_seed(0)
    X = torch.rand(64, 784)
    Y = torch.randint(0, 10, (64,))
    ref = MLP(seed=1)
    opt = torch.optim.SGD(ref.parameters(), 0.1)
    for _ in range(3):
        opt.zero_grad()
        torch.nn.functional.cross_entropy(ref(X), Y).backward()
        opt.step()
    for i, p in enumerate(ref.parameters()):
        a = torch.from_numpy(res[0][1][i])
        for r in range(1, ws):
            assert torch.equal(a, torch.from_numpy(res[r][1][i]))
        assert torch.allclose(a, p.detach(), atol=1e-5)


def test_cluster_ps_worker_example(tmp_path):
    """examples/mnist_example.py as 1 ps + 2 workers on CPU/gloo."""
    p = _free_port()
    hosts = [f"--ps_hosts=127.0.0.1:{p}", f"--worker_hosts=127.0.0.1:{_free_port()},127.0.0.1:{_free_port()}"]
    # the chief's address must be the port we own: pick again if collided
    common = hosts + ["--max_steps=60", "--train_size=3000", "--frequency=20", f"--logs_path={tmp_path}/logs",
                      "--learning_rate=0.05"]
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
    assert r0["global_step"] == 60 and r1["global_step"] == 60
    assert r0["param_sums"] == r1["param_sums"] and r0["param_abs"] == r1["param_abs"]   # lock-step replicas
    assert "Step: 20,  Global Step: 20" in outs["w0"]
    assert "Test-Accuracy:" in outs["w0"] and "ps 0 done" in outs["ps"]
    assert os.listdir(tmp_path / "logs" / "worker_0")


class _FakeBuf:
    def __init__(self, nbytes, ws, rank, fail_alloc, fail_open):
        if fail_alloc:
            raise RuntimeError("hipExtMallocWithFlags failed (simulated)")
        self.fail_open, self.closed = fail_open, False

    def handle(self):
        return b"h" * 8

    def open(self, handles):
        if self.fail_open:
            raise RuntimeError("hipIpcOpenMemHandle failed (simulated)")

    def close(self):
        self.closed = True


def _ipc_setup_worker(rank, ws, port, q, bad_rank, how):
    try:
        sys.path.insert(0, REPO)
        _env(rank, ws, port)
        from distributed_tensorflow_example_amd.parallel import world as W

        w = W.init(backend="gloo")

        class C:
            @staticmethod
            def IpcPeerBuffers(nbytes, ws_, r_):
                return _FakeBuf(nbytes, ws_, r_, how == "alloc" and r_ == bad_rank, how == "open" and r_ == bad_rank)

        try:
            W.open_peer_buffers(C, 1024, w)
            res = "ok"
        except RuntimeError:
            res = "raised"
        # the fallback path after it must still line up collectively on every rank
        assert w.host_all_reduce(1.0, "sum") == ws
        q.put((rank, res))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


@pytest.mark.parametrize("how", ["none", "alloc", "open"])
def test_open_peer_buffers_fails_collectively(how):
    """IPC setup failing on ONE rank (allocation or mapping) makes EVERY rank raise,
    with no rank stuck in the handle exchange (the bench's fallback chain relies on it)."""
    ws, port = 3, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_ipc_setup_worker, args=(r, ws, port, q, 1, how)) for r in range(ws)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(ws))
    for p in ps:
        p.join(timeout=60)
    want = "ok" if how == "none" else "raised"
    assert all(v == want for v in res.values()), res


def test_auto_bucket_mb_cost_model():
    """xGMI bucket sizing (ddp.auto_bucket_mb): k = sqrt(S / (alpha * bw)) buckets."""
    from distributed_tensorflow_example_amd.parallel.ddp import auto_bucket_mb

    bert_bf16 = 110_000_000 * 2
    assert auto_bucket_mb(bert_bf16, 1) == 256.0                 # no comm: one big bucket
    sizes = [auto_bucket_mb(bert_bf16, n) for n in (2, 4, 8)]
    assert all(4.0 <= s <= 256.0 for s in sizes)
    assert sizes == sorted(sizes)                              # more hops -> fewer, larger buckets
    n_buckets = bert_bf16 / 2**20 / sizes[-1]
    assert 3 <= round(n_buckets) <= 8
    assert auto_bucket_mb(1000, 8) == 4.0                      # tiny models clamp at the floor
    # slower hops favour fewer buckets
    assert auto_bucket_mb(bert_bf16, 8, hop_us=30.0) > sizes[-1]
