"""Counter-based normal init (ops.philox_normal_, csrc/kernels/random.hip):
Philox4x32-10 against the Random123 known-answer vectors, Box-Muller moments,
and the sharding invariance the sharded tables rely on (CPU path)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def test_philox4x32_10_known_answers():
    from distributed_tensorflow_example_amd.ops import philox4x32_10

    kat = [((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
           ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
           ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
            (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1))]
    for ctr, key, want in kat:
        got = philox4x32_10(*[np.array([c], np.uint64) for c in ctr], *key)
        assert tuple(int(g[0]) for g in got) == want


def test_normal_moments_and_sharding_invariance():
    from distributed_tensorflow_example_amd.ops import philox_normal_

    full = philox_normal_(torch.empty(100_000, 3), 1, 0, seed=7, mean=0.5, stddev=2.0)
    v = full.numpy().reshape(-1)
    assert abs(v.mean() - 0.5) < 0.03 and abs(v.std() - 2.0) < 0.03
    assert np.isfinite(v).all()
    # rank r of W holds global rows r, r+W, ...: the same values as the full table
    for W in (2, 3):
        for r in range(W):
            n = (100_000 - r + W - 1) // W
            shard = philox_normal_(torch.empty(n, 3), W, r, seed=7, mean=0.5, stddev=2.0)
            assert torch.equal(shard, full[r::W])
    other = philox_normal_(torch.empty(10, 3), 1, 0, seed=8)
    assert not torch.equal(other, philox_normal_(torch.empty(10, 3), 1, 0, seed=7))
