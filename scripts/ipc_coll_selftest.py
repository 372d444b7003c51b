"""Self-test of the IPC collectives (csrc/kernels/ipc_coll.hip) through World's
GPU data plane, one process per rank (torchrun).  On a 1-GPU box every rank
shares cuda:0 (the same mapping, flag and slot protocol as over xGMI).

Checks every collective against an exact host-side expectation (sums in rank
order, as the kernels do): all-reduce sum / avg / max / min over f32 / bf16 /
i32 / i64 with odd tails, one- and two-shot, chunked past the slot capacity;
broadcast of an odd-sized byte tensor; all-gather; uneven all-to-all with
4- and 8-byte rows; the fused all-reduce + SGD; and a captured hipGraph of
an all-reduce + all-to-all replayed with new inputs.  Prints one JSON line.

    python -m torch.distributed.run --nproc-per-node 4 --master-addr 127.0.0.1 scripts/ipc_coll_selftest.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("DTF_DATA_PLANE", "ipc")

import torch  # noqa: E402

from distributed_tensorflow_example_amd.parallel import world as world_mod  # noqa: E402


def data(r, n, dtype, seed, dev):
    g = torch.Generator(device="cpu").manual_seed(seed * 1000 + r)
    if dtype in (torch.int32, torch.int64):
        return torch.randint(-1000, 1000, (n,), generator=g, dtype=dtype).to(dev)
    return (torch.randn(n, generator=g) * (r + 1)).to(dtype).to(dev)


def expect_reduce(W, n, dtype, seed, op, dev):
    xs = [data(r, n, dtype, seed, dev) for r in range(W)]
    if op in ("sum", "avg"):
        acc = xs[0].float() if dtype == torch.bfloat16 else xs[0].clone()
        for x in xs[1:]:
            acc = acc + (x.float() if dtype == torch.bfloat16 else x)
        if op == "avg":
            acc = acc * torch.tensor(1.0 / W, dtype=torch.float32)
        return acc.to(dtype)
    acc = xs[0].clone()
    for x in xs[1:]:
        acc = torch.maximum(acc, x) if op == "max" else torch.minimum(acc, x)
    return acc


def fault_run(w):
    """The last rank skips one all-reduce: every other rank's kernel must give
    up after DTF_IPC_TIMEOUT_S, raise its error word, and the next call on
    that rank must raise instead of hanging."""
    W, r, dev = w.world_size, w.rank, w.device
    t = torch.ones(1024, device=dev)
    w.all_reduce(t, "sum")                     # the plane is up on every rank
    torch.cuda.synchronize()
    if r != W - 1:
        w.all_reduce(t, "sum")                 # its peer never arrives
    torch.cuda.synchronize()                   # the waiting ranks return after their timeout
    err = int(w.ipc.error())
    w.barrier()                                # (gloo) the last rank issues nothing before this
    raised = False
    if r != W - 1:
        try:
            w.all_reduce(t, "sum")
        except RuntimeError:
            raised = True
    torch.cuda.synchronize()
    states = [tuple(x) for x in w.all_gather_object((err, raised))]
    ok = all(e == 1 and rz for e, rz in states[:-1]) and states[-1] == (0, False)
    if r == 0:
        print(json.dumps({"ipc_coll_fault": "pass" if ok else "fail", "states": states}), flush=True)
    return 0 if ok else 1


def main():
    w = world_mod.init(backend="rccl", rccl="lazy")
    if "--fault" in sys.argv:
        return fault_run(w)
    W, r, dev = w.world_size, w.rank, w.device
    fails = []

    def check(name, got, want, rtol=0.0):
        if rtol and got.shape == want.shape:
            err = (got.float().cpu() - want.float().cpu()).abs().max().item()
            if err > rtol * max(want.float().abs().max().item(), 1e-30):
                fails.append(f"{name}: max diff {err}")
            return
        if not torch.equal(got.cpu(), want.cpu()):
            d = (got.float() - want.float()).abs().max().item() if got.shape == want.shape else "shape"
            fails.append(f"{name}: max diff {d}")

    cases = [(1_000_003, torch.float32, "sum"), (999, torch.float32, "avg"), (4097, torch.bfloat16, "sum"),
             (3, torch.bfloat16, "sum"), (70_001, torch.int64, "max"), (12_345, torch.int32, "min"),
             (300_000, torch.float32, "avg"), (5, torch.float64, "sum")]
    for i, (n, dt, op) in enumerate(cases):
        t = data(r, n, dt, i, dev)
        w.all_reduce(t, op)
        check(f"all_reduce[{n},{dt},{op}]", t, expect_reduce(W, n, dt, i, op, dev))
    # chunked: more than one slot's worth (the test sets DTF_IPC_SLOT_MB small)
    cap = w.ipc.capacity()
    n = cap // 4 * 2 + 7
    t = data(r, n, torch.float32, 99, dev)
    w.all_reduce(t, "sum")
    check("all_reduce[chunked]", t, expect_reduce(W, n, torch.float32, 99, "sum", dev))

    # broadcast of an odd-sized byte tensor from rank 1 (padded through a temp)
    src = 1 % W
    b = torch.arange(1001, dtype=torch.int64).remainder(251).to(torch.uint8).to(dev) if r == src else \
        torch.zeros(1001, dtype=torch.uint8, device=dev)
    w.broadcast(b, src)
    check("broadcast[u8]", b, torch.arange(1001, dtype=torch.int64).remainder(251).to(torch.uint8))
    f = data(r, 33, torch.float32, 7, dev)
    w.broadcast(f, 0)
    check("broadcast[f32]", f, data(0, 33, torch.float32, 7, dev))

    # all-gather
    x = data(r, 513, torch.float32, 11, dev)
    out = torch.empty(W * 513, device=dev)
    w.all_gather(x, out)
    check("all_gather", out, torch.cat([data(q, 513, torch.float32, 11, dev) for q in range(W)]))

    # uneven all-to-all: rank q sends (q + d + 1) rows to destination d
    for cols, dt in ((3, torch.int64), (5, torch.float32)):
        send = [q + d + 1 for q in (r,) for d in range(W)]
        recv = [q + r + 1 for q in range(W)]
        rows = sum(send)
        s = (torch.arange(rows * cols, dtype=torch.float64).view(rows, cols) + 1000 * r).to(dt).to(dev)
        d = torch.full((sum(recv), cols), -1, dtype=dt, device=dev)
        w.all_to_all(s, send, d, recv)
        parts = []
        for q in range(W):
            sq = (torch.arange(sum(q + e + 1 for e in range(W)) * cols, dtype=torch.float64).view(-1, cols)
                  + 1000 * q).to(dt)
            off = sum(q + e + 1 for e in range(r))
            parts.append(sq[off:off + q + r + 1])
        check(f"all_to_all[{cols},{dt}]", d, torch.cat(parts))

    # fused all-reduce mean + SGD (3 parameters, odd total)
    shapes = [(7, 3), (5,), (2, 2)]
    ps = [data(0, int(torch.tensor(sh).prod()), torch.float32, 40 + k, dev).view(sh) for k, sh in enumerate(shapes)]
    n = sum(p.numel() for p in ps)
    grad = torch.zeros(n + 1, device=dev)
    grad[:n] = data(r, n, torch.float32, 50, dev)
    gs = torch.zeros(1, dtype=torch.int64, device=dev)
    want_p = torch.cat([p.reshape(-1) for p in ps]).clone()
    gsum = data(0, n, torch.float32, 50, dev)
    for q in range(1, W):
        gsum = gsum + data(q, n, torch.float32, 50, dev)
    lr = 0.25
    step = torch.tensor(lr, dtype=torch.float32) * torch.tensor(1.0 / W, dtype=torch.float32)
    want_p = want_p - step.to(dev) * gsum
    w.ipc.reduce_sgd(grad, ps, lr_val=lr, gstep=gs)
    check("reduce_sgd", torch.cat([p.reshape(-1) for p in ps]), want_p, rtol=1e-6)   # (fma contraction)
    check("reduce_sgd[gstep]", gs, torch.ones(1, dtype=torch.int64))

    # captured hipGraph: all-reduce + all-to-all replayed with new inputs (device sequence numbers)
    n = 2048
    xin = torch.zeros(n, device=dev)
    sa = torch.zeros(W * 4, 2, device=dev)
    sd = torch.zeros(W * 4, 2, device=dev)
    torch.cuda.synchronize()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(st):
        w.all_reduce(xin, "sum")          # warm (first call on this stream)
        w.all_to_all(sa, [4] * W, sd, [4] * W)
        with torch.cuda.graph(g, stream=st):
            w.all_reduce(xin, "sum")
            w.all_to_all(sa, [4] * W, sd, [4] * W)
    torch.cuda.current_stream().wait_stream(st)
    for it in range(3):
        xin.copy_(data(r, n, torch.float32, 200 + it, dev))
        sa.copy_(torch.arange(W * 8, dtype=torch.float32, device=dev).view(W * 4, 2) + 100 * r + it)
        g.replay()
        torch.cuda.synchronize()
        check(f"graph[{it}].all_reduce", xin, expect_reduce(W, n, torch.float32, 200 + it, "sum", dev))
        want = torch.cat([(torch.arange(W * 8, dtype=torch.float32).view(W * 4, 2) + 100 * q + it)[4 * r:4 * r + 4]
                          for q in range(W)])
        check(f"graph[{it}].all_to_all", sd, want)

    torch.cuda.synchronize()
    err = w.ipc.error()
    if err:
        fails.append(f"ipc error word {err}")
    allf = w.all_gather_object(fails)
    res = {"ipc_coll_selftest": "pass" if not any(allf) else "fail", "world_size": W, "rank": r,
           "calls": int(w.ipc.calls()), "rccl_comm": w.comm is not None, "fails": allf}
    if r == 0:
        print(json.dumps(res), flush=True)
    w.barrier()
    return 0 if not any(allf) else 1


if __name__ == "__main__":
    sys.exit(main())
