"""Dropout seed convention (ops/transformer.py next_seed): bit 63 selects the
32-bit hash in every mask-regenerating kernel (csrc/kernels/common.h hash32);
seeds cross into C++ as int64, so a flagged seed is a negative Python int with
the same bits.  DTF_DROPOUT_HASH=64 keeps the splitmix64 hash (bit 63 clear)."""
import importlib
import os

import pytest


def _fresh(env):
    old = os.environ.get("DTF_DROPOUT_HASH")
    try:
        if env is None:
            os.environ.pop("DTF_DROPOUT_HASH", None)
        else:
            os.environ["DTF_DROPOUT_HASH"] = env
        from distributed_tensorflow_example_amd.ops import transformer as T
        return importlib.reload(T)
    finally:
        if old is None:
            os.environ.pop("DTF_DROPOUT_HASH", None)
        else:
            os.environ["DTF_DROPOUT_HASH"] = old


@pytest.mark.parametrize("env,flag", [(None, 1), ("32", 1), ("64", 0)])
def test_seed_bit63_selects_hash(env, flag):
    T = _fresh(env)
    T.set_dropout_seed(7)
    seeds = [T.next_seed() for _ in range(64)]
    for s in seeds:
        assert -(1 << 63) <= s < (1 << 63)                  # fits int64 (pybind int64_t)
        assert ((s & ((1 << 64) - 1)) >> 63) == flag        # bit 63 as the kernels see it
    assert len(set(seeds)) == len(seeds)                    # distinct per call
    T.set_dropout_seed(7)
    assert [T.next_seed() for _ in range(64)] == seeds      # reproducible from the base seed
    _fresh(None)
