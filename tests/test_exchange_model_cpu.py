"""Host-side emulation of the persistent engine's N-GPU exchange layout
(scripts/exchange_cost_model.py mirrors csrc/kernels/mlp_persist_f32.hip):
at every W = 2..8 each dW1 element travels in exactly one lane entry, the
two-shot chunks (wave w -> owner w % W) partition the slot, and the bytes on
the wire are the payload -- no padding."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
import exchange_cost_model as M  # noqa: E402


@pytest.mark.parametrize("bf16", [True, False])
def test_every_dw1_element_in_exactly_one_entry(bf16):
    seen = {}
    for j in range(M.NJ):
        for q in range(M.NQ):
            for w in range(M.NW_WAVES):
                for lane in range(M.LANES):
                    _, elems = M.lane_entries(j, q, w, lane, bf16)
                    for e in elems:
                        assert e not in seen, (e, seen[e], (j, q, w, lane))
                        seen[e] = (j, q, w, lane)
    assert len(seen) == M.DIN * M.HID
    assert all(0 <= f < M.DIN and 0 <= h < M.HID for f, h in seen)


@pytest.mark.parametrize("W", range(2, 9))
def test_two_shot_chunks_partition_every_slot(W):
    owners = {w: w % W for w in range(M.NW_WAVES)}
    for r in range(W):
        own = [w for w in range(M.NW_WAVES) if owners[w] == r]
        foreign = [w for w in range(M.NW_WAVES) if owners[w] != r]
        assert sorted(own + foreign) == list(range(M.NW_WAVES))
        for j in range(M.NJ):
            for q in range(M.NQ):
                assert M.slot_bytes(j, q, True, own) + M.slot_bytes(j, q, True, foreign) == M.slot_bytes(j, q, True)
    # the small part (dW2 / db1 / db2) rides with wave 7: owned by exactly one rank
    assert sum(1 for r in range(W) if owners[7] == r) == 1


@pytest.mark.parametrize("bf16", [True, False])
@pytest.mark.parametrize("W", [2, 4, 8])
def test_one_shot_wire_bytes_equal_the_payload(W, bf16):
    b = M.per_gpu_remote_bytes(W, "one-shot", bf16)
    assert b == (W - 1) * M.payload_bytes(bf16)
    # dW1 share is exactly 784 x 100 elements of the payload dtype per peer
    dw1 = sum(M.lane_entries(j, q, w, lane, bf16)[0] for j in range(M.NJ) for q in range(M.NQ)
              for w in range(M.NW_WAVES) for lane in range(M.LANES))
    assert dw1 == M.DIN * M.HID * (2 if bf16 else 4)


def test_padding_gone_versus_round_two():
    for W in (2, 4, 8):
        assert M.per_gpu_remote_bytes(W, "one-shot", True) < 0.4 * M.round2_bytes(W, "one-shot", True)
    # W = 8 two-shot moves ~2 (W-1)/W of one payload, not W-1 payloads
    b = M.per_gpu_remote_bytes(8, "two-shot", True)
    assert b < 2.0 * M.payload_bytes(True)
