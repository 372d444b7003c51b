"""Native RcclComm reduction ops on cuda:0 (world 1: every op is the identity,
which pins that the op is accepted by RCCL and wired through the binding).
DDP's fp32 buckets rely on "avg" (ncclAvg) to fold the 1/N average into the
reduction (parallel/ddp.py _launch)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("op", ["sum", "avg", "max", "min"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_rccl_world1_ops_identity(native, op, dtype):
    comm = native.RcclComm(native.rccl_unique_id(), 1, 0)
    t = torch.randn(4099, device="cuda").to(dtype)
    ref = t.clone()
    comm.all_reduce(t, op)
    torch.cuda.synchronize()
    assert torch.equal(t, ref)
