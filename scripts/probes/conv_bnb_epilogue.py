"""ResNet-50 (B=128) conv1 input gradients with the residual BatchNorm's
backward in the epilogue (csrc/kernels/conv_igemm.hip EPI 3) vs the unfused
chain: the dx GEMM accumulating onto the folded residual gradient (in-tree
implicit GEMM / gemm_big / hipBLASLt) + bn.hip's partials pass (dy, x, res
read, g written).  Also the plain BN + ReLU form (EPI 2, conv3's input
gradient).  us per call; effective HBM TB/s of the fused kernel.  One JSON
line per shape.

    python scripts/probes/conv_bnb_epilogue.py [batch]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from distributed_tensorflow_example_amd import _native
    from distributed_tensorflow_example_amd.ops import big_gemm, conv

    C_ = _native.load()
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    cl = torch.channels_last
    # (dy channels = conv1 width, dx channels = block width * 4, spatial)
    for Kd, Cx, H in ((64, 256, 56), (128, 512, 28), (256, 1024, 14), (512, 2048, 7)):
        g = torch.Generator(device="cuda").manual_seed(Kd)
        dy = torch.randn(B, Kd, H, H, device="cuda", generator=g).bfloat16().contiguous(memory_format=cl)
        w = (torch.randn(Kd, Cx, 1, 1, device="cuda", generator=g) * 0.05).bfloat16().contiguous(memory_format=cl)
        x = torch.randn(B, Cx, H, H, device="cuda", generator=g).bfloat16().contiguous(memory_format=cl)
        res = torch.randn_like(x)
        extra = torch.randn_like(x)
        stats = torch.cat([torch.zeros(Cx), torch.ones(Cx), torch.ones(Cx), torch.zeros(Cx)]).cuda()
        wt = torch.empty((Cx, Kd, 1, 1), device="cuda", dtype=torch.bfloat16, memory_format=cl)
        C_.conv3x3_wflip(w, wt)
        P = conv.conv3x3_stat_rows(dy, 1)
        part = torch.empty(2, P, Cx, device="cuda")
        r = {"dy_ch": Kd, "dx_ch": Cx, "H": H}
        for bn in (64, 128):
            r[f"epi3_bn{bn}_us"] = round(big_gemm._time(
                lambda: C_.conv3x3_fwd(dy, wt, extra, part, 1, bn, True, x, stats, res), reps=10) * 1e3, 1)
            r[f"epi2_bn{bn}_us"] = round(big_gemm._time(
                lambda: C_.conv3x3_fwd(dy, wt, extra, part, 1, bn, False, x, stats), reps=10) * 1e3, 1)
            r[f"acc_bn{bn}_us"] = round(big_gemm._time(
                lambda: C_.conv3x3_fwd(dy, wt, extra, None, 1, bn, True), reps=10) * 1e3, 1)
        nbytes = x.numel() * 2 * 4 + dy.numel() * 2
        r["epi3_best_TBps"] = round(nbytes / (min(r["epi3_bn64_us"], r["epi3_bn128_us"]) * 1e-6) / 1e12, 2)
        dy2, w2, ex2 = dy.permute(0, 2, 3, 1).reshape(-1, Kd), w.view(Kd, Cx), extra.permute(0, 2, 3, 1).reshape(-1, Cx)
        r["acc_hipblaslt_us"] = round(big_gemm._time(lambda: ex2.addmm_(dy2, w2), reps=10) * 1e3, 1)
        r["acc_gemm_big_us"] = round(big_gemm._time(
            lambda: C_.gemm_big(dy2, False, w2, False, ex2, beta=1.0), reps=10) * 1e3, 1)
        gamma = torch.ones(Cx, device="cuda")
        coef = torch.empty(3 * Cx, device="cuda")
        dx = torch.empty_like(x)
        dres = torch.empty_like(x)
        dg, db = torch.empty(Cx, device="cuda"), torch.empty(Cx, device="cuda")
        bpart = torch.empty(2 * C_.bn_partial_rows(x.numel() // Cx, Cx) * Cx, device="cuda")
        r["bn_bwd_res_unfused_us"] = round(big_gemm._time(
            lambda: C_.bn_bwd(extra, x, res, gamma, stats, bpart, coef, dx, dres, dg, db, True, False), reps=10) * 1e3, 1)
        r["bn_bwd_parts_us"] = round(big_gemm._time(
            lambda: C_.bn_bwd_parts(extra, x, gamma, stats, part, P, coef, dx, dg, db, False), reps=10) * 1e3, 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
