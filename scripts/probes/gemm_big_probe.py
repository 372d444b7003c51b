"""One gemm_big product repeated (for rocprofv3 PMC passes): role fwd|dx|dw."""
import sys

import torch

sys.path.insert(0, ".")
from distributed_tensorflow_example_amd import _native  # noqa: E402

role = sys.argv[1] if len(sys.argv) > 1 else "fwd"
T, O, I = 16384, 3072, 768
C = _native.load()
bf = torch.bfloat16
x = torch.randn(T, I, device="cuda", dtype=bf)
w = torch.randn(O, I, device="cuda", dtype=bf)
gy = torch.randn(T, O, device="cuda", dtype=bf)
for _ in range(20):
    if role == "fwd":
        C.gemm_big(x, False, w, True, torch.empty(T, O, device="cuda", dtype=bf))
    elif role == "dx":
        C.gemm_big(gy, False, w, False, torch.empty(T, I, device="cuda", dtype=bf))
    else:
        C.gemm_big(gy, True, x, False, torch.zeros(O, I, device="cuda"), beta=1.0)
torch.cuda.synchronize()
