#!/usr/bin/env python3
"""Per-step cost model of the persistent MLP engine's N-GPU gradient exchange
(csrc/kernels/mlp_persist_f32.hip, MULTI section) -- a host-side emulation of
the kernel's slot layout, used both to price the exchange and (tests/
test_exchange_model_cpu.py) to prove the W = 2..8 indexing covers every
gradient element exactly once.

Layout mirrored from the kernel:
  * 28 compute workgroups c = (j, q): hidden block j (16 units, 7 blocks, units
    >= 100 are padding), feature slice q (13, 12, 12, 12 tiles of 16 features).
  * wave w (8 per workgroup) owns local tiles w and w + 8 of its slice; lane
    (r = lane & 15, g = lane >> 4) holds dW1[16 t + 4 g + i][16 j + r], i < 4.
  * bf16 payload: a lane's two tiles in ONE 16-B entry (8 B when the wave has
    one tile); fp32: one 16-B entry per tile.  Lanes of padding units (hv
    false) neither store nor load.
  * wave 7 also carries dW2[16 j + 4 g + i][class r] (16 B, lanes r < 10 with a
    valid unit) and db1 / db2 (4 B, lanes < 16 with a valid unit / 16..25).
  * one-shot: every workgroup reads its slot from each of the W - 1 peers;
    two-shot: wave w's entries form chunk w % W, reduced by its owner, then
    every rank reads each foreign chunk's sums from the owner (bf16 sums for a
    bf16 payload).

Usage: python scripts/exchange_cost_model.py [--json]
"""
from __future__ import annotations

import argparse
import json

DIN, HID, NCLS = 784, 100, 10
NJ, NQ, NW_WAVES, LANES = 7, 4, 8, 64


def ntile(q: int) -> int:
    return 13 if q == 0 else 12


def tile0(q: int) -> int:
    return 0 if q == 0 else 13 + 12 * (q - 1)


def lane_entries(j: int, q: int, w: int, lane: int, bf16: bool):
    """(bytes this lane puts on the wire for its dW1 entries, [(feature, unit), ...] it carries)."""
    r, g = lane & 15, lane >> 4
    hid = 16 * j + r
    if hid >= HID:
        return 0, []
    tiles = [t for t in (w, w + 8) if t < ntile(q)]
    elems = [(16 * (tile0(q) + t) + 4 * g + i, hid) for t in tiles for i in range(4)]
    nbytes = (8 * len(tiles)) if bf16 else (16 * len(tiles))
    return nbytes, elems


def small_bytes(j: int, lane: int) -> int:
    """wave 7's dW2 entry + db1/db2 word of this lane."""
    r, g = lane & 15, lane >> 4
    b = 16 if (r < NCLS and 16 * j + 4 * g < HID) else 0
    b += 4 if (16 * j + lane < HID if lane < 16 else lane < 16 + NCLS) else 0
    return b


def slot_bytes(j: int, q: int, bf16: bool, waves=None) -> int:
    """Payload bytes of workgroup (j, q)'s slot (optionally only `waves`)."""
    tot = 0
    for w in (range(NW_WAVES) if waves is None else waves):
        for lane in range(LANES):
            tot += lane_entries(j, q, w, lane, bf16)[0]
            if w == 7:
                tot += small_bytes(j, lane)
    return tot


def per_gpu_remote_bytes(W: int, mode: str, bf16: bool) -> int:
    """Bytes one GPU reads from its peers per step (== bytes it sends, by symmetry)."""
    if W == 1:
        return 0
    tot = 0
    for j in range(NJ):
        for q in range(NQ):
            if mode == "one-shot":
                tot += (W - 1) * slot_bytes(j, q, bf16)
            else:
                # rank 0's view (the busiest: it owns chunk 0, and wave 0 of a slice
                # always has two tiles).  reduce-scatter: the chunks it owns, from
                # W - 1 peers; all-gather: the chunks it does not own, from their
                # owner (bf16 sums for a bf16 payload)
                own = [w for w in range(NW_WAVES) if w % W == 0]
                foreign = [w for w in range(NW_WAVES) if w % W != 0]
                tot += (W - 1) * slot_bytes(j, q, bf16, own) + slot_bytes(j, q, bf16, foreign)
    return tot


def payload_bytes(bf16: bool) -> int:
    """The gradient itself: dW1 (784 x 100) in the payload dtype + dW2 / db1 / db2 in
    fp32 as the kernel sends them (each slice of a block carries the block's copy)."""
    dw1 = DIN * HID * (2 if bf16 else 4)
    small = sum(small_bytes(j, lane) for j in range(NJ) for lane in range(LANES)) * NQ
    return dw1 + small


def model(W: int, mode: str, bf16: bool, link_gbs: float = 64.0, links: int = 7, hop_us: float = 1.5):
    """Bytes per GPU and a latency-bandwidth estimate of the exchange's step cost.
    link_gbs: sustained peer-read bandwidth of one xGMI link (an estimate; gpurun
    gives one GPU); peers are spread over min(W - 1, links) links; one flag round
    trip per hop (one-shot: 1 hop, two-shot: 2)."""
    b = per_gpu_remote_bytes(W, mode, bf16)
    if W == 1:
        return dict(W=W, mode=mode, payload="bf16" if bf16 else "fp32", bytes_per_gpu=0, est_us=0.0)
    bw = link_gbs * min(W - 1, links) * 1e3        # bytes per us
    hops = 1 if mode == "one-shot" else 2
    return dict(W=W, mode=mode, payload="bf16" if bf16 else "fp32", bytes_per_gpu=b,
                bytes_over_payload_x_peers=round(b / (payload_bytes(bf16) * (W - 1)), 4),
                est_us=round(hops * hop_us + b / bw, 2))


def round2_bytes(W: int, mode: str, bf16: bool) -> int:
    """Round-2 layout (for comparison): every lane entry 16 B (bf16 used 8 of them),
    two entries per lane whatever the tile count, padding lanes loaded too."""
    slot = NW_WAVES * 2 * LANES * 16 + LANES * 16 + (16 + NCLS) * 4
    if mode == "one-shot":
        return (W - 1) * NJ * NQ * slot
    return 2 * (W - 1) * NJ * NQ * slot // W


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    rows = []
    for bf16 in (True, False):
        for mode in ("one-shot", "two-shot"):
            for W in (2, 4, 8):
                m = model(W, mode, bf16)
                m["round2_bytes_per_gpu"] = round2_bytes(W, mode, bf16)
                rows.append(m)
    if a.json:
        print(json.dumps({"payload_bytes_bf16": payload_bytes(True), "payload_bytes_fp32": payload_bytes(False),
                          "rows": rows}, indent=1))
        return
    print(f"gradient payload per rank: bf16 {payload_bytes(True)} B, fp32 {payload_bytes(False)} B")
    print(f"{'payload':7s} {'mode':9s} {'W':>2s} {'bytes/GPU/step':>15s} {'round-2':>10s} {'x(W-1)payload':>14s} {'est us':>7s}")
    for m in rows:
        print(f"{m['payload']:7s} {m['mode']:9s} {m['W']:2d} {m['bytes_per_gpu']:15d} {m['round2_bytes_per_gpu']:10d} "
              f"{m.get('bytes_over_payload_x_peers', 0):14.3f} {m['est_us']:7.2f}")


if __name__ == "__main__":
    main()
