"""Phase timing of the fp32 persistent MLP kernel (csrc/kernels/mlp_persist_f32.hip)
from in-kernel s_memrealtime stamps (100 MHz).

Stamps per step (workgroup c, wave 0, lane 0): 0 step start, 1 forward MFMAs
done, 2 after LDS barrier A, 3 E1 published, 4 E1 flags matched, 5 z summed,
6 E2 published, 7 E2 flags matched, 8 logits summed, 9 head done, 10 after LDS
barrier B, 11 weight-gradient MFMAs done, 12 update done.
Prints the median / p90 of every segment over steps 1..63 and all compute
workgroups, plus per-step time and launch-level timing.
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from distributed_tensorflow_example_amd.data.mnist import PinnedEpoch, synthetic_mnist  # noqa: E402
from distributed_tensorflow_example_amd.models import mlp  # noqa: E402

NAMES = {"fp32": ["fwd_mfma", "barrier_A", "E1_publish", "E1_wait", "E1_load_sum", "P1_logit_publish",
                       "E2_wait", "E2_load_sum", "head", "barrier_B", "wgrad_mfma", "update"]}


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "fp32"
    names = NAMES["fp32" if prec == "fp32-mfma" else prec]
    B, G = 100, 64
    dev = torch.device("cuda", 0)
    imgs, labels = synthetic_mnist(55000, seed=1)
    ep = PinnedEpoch(imgs, labels, B)
    tr = mlp.FusedMLPTrainer(batch_size=B, lr=0.0005, device=dev)
    run = mlp.PersistentMLPRunner(tr, ep, steps_per_launch=550, precision=prec)
    run.prepare(550)
    run.run(550 * 4)
    torch.cuda.synchronize()
    out = {}
    # launch-level: G-step launches back to back, host wall and device per-step stamps
    for g in (20, 64, 550):
        run.prepare(g)
        run.run(g, lookahead=g)
        torch.cuda.synchronize()
        s0 = tr.global_step
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        run.run(g)
        t1.record()
        torch.cuda.synchronize()
        dt = run.step_times_ms(s0, s0 + g) * 1000.0
        out[f"launch_{g}"] = {"event_us": round(t0.elapsed_time(t1) * 1000.0, 2),
                              "sum_step_us": round(float(dt.sum()), 2),
                              "p50_step_us": round(float(np.median(dt)), 3)}
    ts = torch.zeros(65 * 64 * 16, dtype=torch.int64, device=dev)
    run.phase_ts = ts
    run.prepare(G)
    run.run(G, lookahead=G)
    torch.cuda.synchronize()
    run.phase_ts = None
    raw = ts.cpu().numpy().reshape(65, 64, 16)
    if prec in ("fp32", "fp32-mfma"):
        # launch stamps (row 64): compute wg 0 entry, 4 params loaded, 1 census done, 2 first stage read,
        # 3 loop done, 5 written back; copier 28+cid: 0 entry, 1 done. Relative to the earliest entry, us
        L = raw[64].astype(np.float64) * 0.01
        t0 = min(L[:28, 0].min(), L[28:44, 0].min())
        rel = lambda x: round(float(x - t0), 2)
        first_step = raw[0, :28, 0].astype(np.float64) * 0.01
        out["launch_stamps_us"] = {
            "compute_entry_max": rel(L[:28, 0].max()), "param_loads_issued_max": rel(L[:28, 4].max()),
            "census_params_stage_done_max": rel(L[:28, 1].max()), "first_x_read_max": rel(L[:28, 2].max()),
            "step0_start_max": rel(first_step.max()), "loop_done_max": rel(L[:28, 3].max()),
            "written_back_max": rel(L[:28, 5].max()), "copier_entry_max": rel(L[28:44, 0].max()),
            "copier_done_max": rel(L[28:44, 1].max())}
        raw = raw[:64]
    nj, nq = (7, 4) if prec in ("fp32", "fp32-mfma") else (7, 1)
    ns = len(names) + 1
    r = raw[1:G, : nj * nq, :ns].astype(np.float64) * 0.01   # us
    seg = {}
    for k, name in enumerate(names):
        d = r[:, :, k + 1] - r[:, :, k]
        seg[name] = [round(float(np.median(d)), 3), round(float(np.percentile(d, 90)), 3)]
    out["segments_us_median_p90"] = seg
    step = r[1:, :, 0] - r[:-1, :, 0]
    out["step_us_median"] = round(float(np.median(step)), 3)
    pub = 6 if prec in ("fp32", "fp32-mfma") else 3
    got = pub + 1
    last = r[:, :, pub].max(axis=1, keepdims=True)
    hop = r[:, :, got] - last
    out["logit_edge_hop_after_last_publish_us_median_p90"] = [round(float(np.median(hop)), 3),
                                                               round(float(np.percentile(hop, 90)), 3)]
    out["logit_publish_skew_us_median"] = round(float(np.median(r[:, :, pub].max(1) - r[:, :, pub].min(1))), 3)
    if prec in ("fp32", "fp32-mfma"):
        # extra stamps: 13 wave 7 folded the last head tile (dW2 / db / metrics), 14 wave 7 step
        # start, 15 wave 7 saw its next-step stage land (vmcnt(0)) -- then barrier B
        med = lambda x: round(float(np.median(x)), 3)
        rs = raw[1:G, : nj * nq, :].astype(np.float64) * 0.01
        if int(os.environ.get("DTF_PERSIST_DBG", "0")) & 2:
            out["head_detail_us_from_logits_summed"] = {
                "softmax_done": med(rs[:, :, 13] - rs[:, :, 8]), "da_mfma_done": med(rs[:, :, 14] - rs[:, :, 8]),
                "dz2_planes_rowsums_done": med(rs[:, :, 15] - rs[:, :, 8]), "head_done": med(rs[:, :, 9] - rs[:, :, 8])}
        out["barrier_B_detail_us_from_w0_step_start"] = {
            "w7_step_start": med(rs[:, :, 14] - rs[:, :, 0]), "w0_head_done": med(rs[:, :, 9] - rs[:, :, 0]),
            "w7_last_head_folded": med(rs[:, :, 13] - rs[:, :, 0]),
            "w7_stage_landed": med(rs[:, :, 15] - rs[:, :, 0]),
            "barrier_B_exit": med(rs[:, :, 10] - rs[:, :, 0])}
    late = (r[:, :, 0] - r[:, :, 0].min(axis=1, keepdims=True)).mean(axis=0)
    out["step_start_lateness_us_by_wg"] = np.round(late, 2).tolist()
    np.save(os.path.join(REPO, "gpurun_out", f"phase_raw_{prec}.npy"), raw[:G])
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
