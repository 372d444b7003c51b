"""Time the NHWC 3x3 / stride-2 max-pool forward and backward at ResNet-50's
stem shape (B = 128, 112x112x64 bf16, channels_last); prints one JSON line.
DTF_POOL_XCD=0 selects the plain block order (read once per process)."""
import json
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from distributed_tensorflow_example_amd.ops import big_gemm  # noqa: E402
from distributed_tensorflow_example_amd.ops.pool import max_pool2d  # noqa: E402


def main():
    x = torch.randn(128, 64, 112, 112, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    x.requires_grad_()
    y = max_pool2d(x, 3, 2, 1)
    g = torch.randn_like(y)
    fwd = big_gemm._time(lambda: max_pool2d(x, 3, 2, 1), reps=20) * 1e3
    bwd = big_gemm._time(lambda: torch.autograd.grad(y, x, g, retain_graph=True), reps=20) * 1e3
    print(json.dumps({"xcd": os.environ.get("DTF_POOL_XCD", "1"), "fwd_us": round(fwd, 1), "bwd_us": round(bwd, 1)}))


if __name__ == "__main__":
    main()
