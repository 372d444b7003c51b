"""Bucketed, backward-overlapped DDP (parallel/ddp.py) on the GPU with two
ranks sharing cuda:0: gradient-as-bucket-view hooks, the side comm stream and
its events, the fused bf16 / fp16 pack + 1/N kernels around the 16-bit
reduction.  RCCL refuses two ranks on one device, so the reduction under the
comm stream is gloo's (CUDA tensors staged by gloo, ordered on the current
stream) behind RcclComm's all_reduce interface; everything around it is the
code path an 8-GPU node runs.  Result: == full-batch SGD on one rank (fp32),
within 16-bit rounding for bf16 / fp16 communication."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _GlooStreamComm:
    """RcclComm's all_reduce / broadcast over the gloo process group."""

    def all_reduce(self, t, op="sum"):
        import torch.distributed as dist

        dist.all_reduce(t)
        if op == "avg":
            t.div_(dist.get_world_size())

    def broadcast(self, t, src):
        import torch.distributed as dist

        dist.broadcast(t, src)


def _worker(rank, ws, port, q, bucket_mb, comm):
    try:
        sys.path.insert(0, REPO)
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(ws), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(port))
        from distributed_tensorflow_example_amd import optim
        from distributed_tensorflow_example_amd.models.mlp import MLP
        from distributed_tensorflow_example_amd.parallel import world as W
        from distributed_tensorflow_example_amd.parallel.ddp import DistributedDataParallel

        w = W.init(backend="gloo")
        dev = torch.device("cuda", 0)
        w.device = dev
        w.comm = _GlooStreamComm()
        torch.manual_seed(0)
        X = torch.rand(64, 784, device=dev)
        Y = torch.randint(0, 10, (64,), device=dev)
        model = MLP(seed=1 + rank).to(dev)                    # different init: DDP broadcasts rank 0's
        cd = {"fp32": None, "bf16": torch.bfloat16, "fp16": torch.float16}[comm]
        ddp = DistributedDataParallel(model, w, bucket_mb=bucket_mb, comm_dtype=cd)
        assert ddp.comm_stream is not None
        opt = optim.FusedSGD(list(model.parameters()), 0.1)
        shard = slice(rank * 64 // ws, (rank + 1) * 64 // ws)
        for _ in range(3):
            ddp.zero_grad()
            loss = torch.nn.functional.cross_entropy(ddp(X[shard]), Y[shard])
            loss.backward()
            ddp.finish_gradient_synchronization()
            opt.step()
        torch.cuda.synchronize()
        q.put((rank, [p.detach().cpu().numpy().copy() for p in model.parameters()], len(ddp.buckets)))
    except Exception:
        import traceback

        q.put((rank, traceback.format_exc(), 0))


@pytest.mark.parametrize("comm,bucket_mb", [("fp32", 0.001), ("fp32", 25.0), ("bf16", 0.001), ("fp16", 0.001)])
def test_ddp_two_ranks_same_gpu_match_full_batch(comm, bucket_mb):
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q, bucket_mb, comm)) for r in range(ws)]
    [p.start() for p in procs]
    res = sorted([q.get(timeout=150) for _ in range(ws)], key=lambda r: r[0])
    [p.join(60) for p in procs]
    for r in res:
        assert isinstance(r[1], list), r[1]
    if bucket_mb < 1:
        assert res[0][2] > 1                                # really bucketed
    sys.path.insert(0, REPO)
    from distributed_tensorflow_example_amd.models.mlp import MLP

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    X = torch.rand(64, 784, device=dev)
    Y = torch.randint(0, 10, (64,), device=dev)
    ref = MLP(seed=1).to(dev)
    opt = torch.optim.SGD(ref.parameters(), 0.1)
    for _ in range(3):
        opt.zero_grad()
        torch.nn.functional.cross_entropy(ref(X), Y).backward()
        opt.step()
    tol = 1e-5 if comm == "fp32" else 2e-3
    for i, p in enumerate(ref.parameters()):
        a = torch.from_numpy(res[0][1][i])
        assert torch.equal(a, torch.from_numpy(res[1][1][i]))     # replicas stay identical
        assert torch.allclose(a, p.detach().cpu(), atol=tol), (comm, i, float((a - p.detach().cpu()).abs().max()))
