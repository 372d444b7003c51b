"""Phase timing of the persistent MLP kernel from in-kernel s_memrealtime stamps.

Stamps (compute workgroup j, wave 0): 0 step start, 1 forward done, 2 exchange
complete, 3 after S_b (head done), 4 weight-gradient done, 5 after S_a.
Copier workgroups stamp their first and last instruction.  Also times whole
launches with and without the in-kernel input copy.
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


def main():
    B, G = 100, 50  # per-launch stamps cover 50 steps
    dev = torch.device("cuda", 0)
    imgs, labels = synthetic_mnist(55000, seed=1)
    ep = PinnedEpoch(imgs, labels, B)
    tr = mlp.FusedMLPTrainer(batch_size=B, lr=0.0005, device=dev)
    run = mlp.PersistentMLPRunner(tr, ep, steps_per_launch=G)
    run.run(10 * G)
    torch.cuda.synchronize()
    C = tr.C
    ts = torch.zeros(64 * 8 * 16 + 2 * 64, dtype=torch.int64, device=dev)

    def launch(copy: bool, stamps: bool):
        par = run.parity
        nxt = (0, G)
        C.mlp_persist(run.xs[par], run.xts[par], ep.rec, B, G, tr.params, tr.lr, tr.metrics, tr.gstep, run.seq,
                      run.gran, run.err, 5.0, tr.act, 0, host=ep.host, host_offset=0,
                      next_steps=G if copy else 0, xs_next=run.xs[par ^ 1], xts_next=run.xts[par ^ 1],
                      ts=ts if stamps else None)

    out = {}
    for copy in (True, False):
        evs = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            launch(copy, False)
            e1.record()
            evs.append((e0, e1))
        torch.cuda.synchronize()
        ms = [a.elapsed_time(b) for a, b in evs[5:]]
        out[f"launch_us_copy={copy}"] = round(1000 * float(np.median(ms)), 2)
    ts.zero_()
    launch(True, True)
    torch.cuda.synchronize()
    t = ts.cpu().numpy()
    st = t[: 64 * 8 * 16].reshape(64, 8, 16)[:G, :7, :6].astype(np.float64) * 10.0 / 1000.0  # us
    base = st[0, :, 0].min()
    ph = {}
    names = ["fwd", "publish->exchange", "head_rest", "wgrad", "S_a"]
    for k in range(5):
        d = st[1:, :, k + 1] - st[1:, :, k]
        ph[names[k]] = [round(float(np.median(d)), 3), round(float(np.percentile(d, 90)), 3)]
    raw = t[: 64 * 8 * 16].reshape(64, 8, 16)[:G, :7, :]
    pub = (raw[1:, :, 6] - raw[1:, :, 1]).astype(np.float64) * 0.01
    wait = (raw[1:, :, 2] - raw[1:, :, 6]).astype(np.float64) * 0.01
    out["publish_and_lds_writes_us"] = [round(float(np.median(pub)), 3), round(float(np.percentile(pub, 90)), 3)]
    out["spin_us"] = [round(float(np.median(wait)), 3), round(float(np.percentile(wait, 90)), 3)]
    sw = raw[1:, :, 7]
    out["sweeps_median_max"] = [float(np.median(sw)), float(sw.max())]
    # when does the LAST workgroup publish (stamp 1) vs when each finishes its spin (stamp 2)
    last_pub = raw[1:, :, 1].max(axis=1)
    out["last_fwd_done_to_spin_done_us"] = round(float(np.median((raw[1:, :, 2].T - last_pub).T * 0.01)), 3)
    w7a = (raw[1:, :, 9] - raw[1:, :, 8]).astype(np.float64) * 0.01
    w7b = (raw[1:, :, 10] - raw[1:, :, 9]).astype(np.float64) * 0.01
    w7c = (raw[1:, :, 5] - raw[1:, :, 10]).astype(np.float64) * 0.01
    out["wave7_small_params_us"] = round(float(np.median(w7a)), 3)
    out["wave7_wgrad_us"] = round(float(np.median(w7b)), 3)
    out["wave7_publish_to_S_a_exit_us"] = round(float(np.median(w7c)), 3)
    def seg(a_, b_):
        d = (raw[1:, :, b_] - raw[1:, :, a_]).astype(np.float64) * 0.01
        return round(float(np.median(d)), 3)
    out["fwd_plus_wait_small_us"] = seg(0, 13)
    out["payload_return_us"] = seg(2, 11)
    out["softmax_to_S_b_us"] = seg(11, 12)
    out["S_b_wait_us"] = seg(12, 3)
    steps = st[2:, 0, 0] - st[1:-1, 0, 0]
    out["step_us_median"] = round(float(np.median(steps)), 3)
    out["phase_us_median_p90"] = ph
    out["wg_start_skew_us"] = round(float(st[0, :, 0].max() - st[0, :, 0].min()), 3)
    cp = t[64 * 8 * 16:].reshape(64, 2)[:57].astype(np.float64) * 10.0 / 1000.0
    out["copier_window_us"] = [round(float(cp[:, 0].min() - base), 2), round(float(cp[:, 1].max() - base), 2)]
    out["compute_window_us"] = round(float(st[G - 1, :, 5].max() - base), 2)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
