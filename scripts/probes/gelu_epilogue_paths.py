"""Per-call times (us) of BERT-base's FFN-up forward / FFN-down input gradient
with and without the fused GELU epilogues of gemm_big.hip (gemm_gelu_aux,
gemm_dgelu) at T = 16384 tokens, hidden 768, intermediate 3072."""
import json

import torch

from distributed_tensorflow_example_amd import _native
from distributed_tensorflow_example_amd.ops import big_gemm

C = _native.load()
dev = torch.device("cuda")
bf = torch.bfloat16
M, N, K = 16384, 3072, 768
us = lambda f: round(big_gemm._time(f, reps=10) * 1e3, 1)
x, w1 = torch.randn(M, K, device=dev, dtype=bf), torch.randn(N, K, device=dev, dtype=bf)
u, h = torch.empty(M, N, device=dev, dtype=bf), torch.empty(M, N, device=dev, dtype=bf)
b = torch.randn(N, device=dev)
fwd = {"gemm_gelu_aux": us(lambda: C.gemm_gelu_aux(x, False, w1, True, h, u, b)),
       "gemm_big_fwd": us(lambda: C.gemm_big(x, False, w1, True, u)),
       "hipblaslt_fwd": us(lambda: torch.mm(x, w1.t(), out=u)),
       "bias_gelu_fwd": us(lambda: C.bias_gelu_fwd(u, b, h))}
dy, w2 = torch.randn(M, K, device=dev, dtype=bf), torch.randn(K, N, device=dev, dtype=bf)
du, db = torch.empty(M, N, device=dev, dtype=bf), torch.empty(N, device=dev)
colpart, part = torch.empty(M // 128 * N, device=dev), torch.empty(big_gemm.gelu_bwd_slices(M) * N, device=dev)
bwd = {"gemm_dgelu": us(lambda: C.gemm_dgelu(dy, False, w2, False, du, u, b, colpart, db)),
       "gemm_big_dx": us(lambda: C.gemm_big(dy, False, w2, False, h)),
       "hipblaslt_dx": us(lambda: torch.mm(dy, w2, out=h)),
       "bias_gelu_bwd": us(lambda: C.bias_gelu_bwd(h, u, b, du, part, db, accumulate=False))}
print(json.dumps({"shape": [M, N, K], "fwd_us": fwd, "bwd_us": bwd}))
