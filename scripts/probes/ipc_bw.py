"""IPC collectives' per-call time and effective bandwidth (torchrun, ranks on
the visible GPU(s); on a 1-GPU box all ranks share cuda:0 -- peer reads then
come from the same HBM, not over xGMI).  Prints one JSON line (rank 0).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 scripts/probes/ipc_bw.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("DTF_DATA_PLANE", "ipc")

import torch  # noqa: E402

from distributed_tensorflow_example_amd.parallel import world as world_mod  # noqa: E402


def timed(w, fn, reps=20):
    fn()
    torch.cuda.synchronize()
    w.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return w.host_all_reduce(e0.elapsed_time(e1) / reps * 1e3, "max")    # us


def main():
    w = world_mod.init(backend="rccl", rccl="lazy")
    W, dev = w.world_size, w.device
    res = {"world_size": W, "narrow": os.environ.get("DTF_IPC_NARROW", "0") == "1", "ops": {}}
    for mb in (0.3, 1, 8, 32):
        n = int(mb * (1 << 20)) // 4
        t = torch.randn(n, device=dev)
        us = timed(w, lambda: w.all_reduce(t, "sum"))
        res["ops"][f"all_reduce_{mb}MB"] = {"us": round(us, 1), "peer_read_GBps": round((W - 1) * 4 * n / us / 1e3, 1)}
        rows = n // 16
        per = rows // W
        s = torch.randn(per * W, 16, device=dev)
        d = torch.empty_like(s)
        us = timed(w, lambda: w.all_to_all(s, [per] * W, d, [per] * W))
        res["ops"][f"all_to_all_{mb}MB"] = {"us": round(us, 1),
                                            "peer_read_GBps": round((W - 1) * per * 64 / us / 1e3, 1)}
    b = torch.randn(8 << 20, device=dev)
    us = timed(w, lambda: w.broadcast(b, 0))
    res["ops"]["broadcast_32MB"] = {"us": round(us, 1), "GBps": round(32 * (1 << 20) / us / 1e3, 1)}
    x = torch.randn(8 << 20, device=dev)
    y = torch.empty_like(x)
    us = timed(w, lambda: y.copy_(x))
    res["ops"]["local_copy_32MB"] = {"us": round(us, 1)}
    if w.rank == 0:
        print(json.dumps(res), flush=True)
    w.barrier()


if __name__ == "__main__":
    main()
