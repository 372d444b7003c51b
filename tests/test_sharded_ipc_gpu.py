"""The sharded tables' data plane without RCCL: sparse LR (lr2.py's ps-held
W[F, 1], lr2.py:359-396) and Wide&Deep (the deep tower of
lr2_debug.py:423-428) with 2 and 4 ranks sharing cuda:0, every id / row /
gradient exchange (exact-count and static equal-split all-to-all) and every
all-reduce on the IPC collectives (csrc/kernels/ipc_coll.hip): the trained
tables equal one rank on the whole batch, also when every static step
overflows and is voided + replayed exactly.  No RCCL communicator is created."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from test_sparse_cpu import _run, svm_dir  # noqa: E402,F401

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu_ranks(monkeypatch):
    monkeypatch.setenv("DTF_TEST_BACKEND", "rccl")      # every rank on cuda:0, World's GPU data plane
    monkeypatch.setenv("DTF_IPC_TIMEOUT_S", "60")


def _planes(res, ws):
    for r in res:
        p = r[6]
        assert not p["rccl"], p
        assert (p["ipc_calls"] > 0) == (ws > 1), p


@pytest.mark.parametrize("ws", [2, 4])
@pytest.mark.parametrize("kind", ["lr", "lr-static", "wd", "wd-static"])
def test_sharded_tables_on_ipc_equal_one_rank(svm_dir, ws, kind):
    d, tr, te = svm_dir
    lr = 0.2 if kind.startswith("wd") else 0.5
    one = _run(1, tr, 6, lr, kind.split("-")[0])
    many = _run(ws, tr, 6, lr, kind)
    _planes(many, ws)
    assert np.array_equal(one[0][1], many[0][1])                 # init independent of sharding
    for r in range(1, ws):
        assert np.array_equal(many[0][2], many[r][2])            # replicas / shards agree
    assert np.allclose(one[0][2], many[0][2], atol=1e-5), np.abs(one[0][2] - many[0][2]).max()
    if kind.startswith("wd"):
        assert np.allclose(one[0][3], many[0][3], atol=1e-5)     # first tower layer (Adam)
        assert np.allclose(one[0][4], many[0][4], atol=1e-5)     # wide table
    else:
        assert abs(one[0][3] - many[0][3]) < 1e-5
    assert not np.allclose(one[0][1], one[0][2])                 # it trained


@pytest.mark.parametrize("kind", ["lr", "wd"])
def test_overflow_voiding_on_ipc_equal_one_rank(svm_dir, kind):
    d, tr, te = svm_dir
    lr = 0.2 if kind == "wd" else 0.5
    one = _run(1, tr, 6, lr, kind)
    four = _run(4, tr, 6, lr, kind + "-static", 1)
    _planes(four, 4)
    for r in range(1, 4):
        assert np.array_equal(four[0][2], four[r][2])
    st = four[0][5]
    assert st["voided"] == 6 and st["gstep"] == 6, st
    assert np.allclose(one[0][2], four[0][2], atol=1e-5)
