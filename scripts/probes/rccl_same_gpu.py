"""Can RCCL run a 2-rank communicator with both ranks on cuda:0 (the only way
to execute RCCL at world > 1 on a 1-GPU box)?  Launch under
torch.distributed.run --nproc-per-node 2; prints one JSON line from rank 0."""
import json
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
out = {"rank": rank}
try:
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    t = torch.full((1 << 20,), float(rank + 1), device="cuda")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    out["allreduce_ok"] = bool(torch.all(t == 3.0).item())
    dist.destroy_process_group()
except Exception as e:  # noqa: BLE001
    out["error"] = repr(e)[:400]
if rank == 0:
    print(json.dumps(out), flush=True)
