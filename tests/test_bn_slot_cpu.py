"""CPU checks of the host-side logic around the BN-backward conv epilogues
(ops/bn.py BwdSlot, ops/conv.py _bnb_fits / _fuse_bnb) and the one flat DDP
gradient buffer (parallel/ddp.py): the GPU tests cover the kernels, these pin
the decisions that route a gradient onto them."""
import pytest
import torch


class _T:
    """A stand-in for a tensor's metadata (data_ptr / _version / shape)."""

    def __init__(self, ptr, ver=0, shape=(2, 8, 4, 4)):
        self._ptr, self._version, self.shape = ptr, ver, torch.Size(shape)

    def data_ptr(self):
        return self._ptr


def test_bwd_slot_take_requires_the_untouched_conv_gradient():
    from distributed_tensorflow_example_amd.ops.bn import BwdSlot

    s = BwdSlot(x=None, stats=None)
    assert s.take(_T(1)) is None                       # no partials written
    g = _T(7, ver=3)
    s.part, s.g, s.g_version = ("part", 5), g, 3
    assert s.take(_T(8, ver=3)) is None                # another tensor (e.g. autograd summed two branches)
    assert s.part is None                              # taking clears the slot either way
    s.part, s.g, s.g_version = ("part", 5), g, 3
    assert s.take(_T(7, ver=4)) is None                # same storage, modified in place since
    s.part, s.g, s.g_version = ("part", 5), g, 3
    assert s.take(_T(7, ver=3, shape=(2, 8, 4, 2))) is None
    s.part, s.g, s.g_version = ("part", 5), g, 3
    assert s.take(_T(7, ver=3)) == ("part", 5)


def test_bnb_fits_plain_and_residual_forms():
    from distributed_tensorflow_example_amd.ops.bn import BwdSlot
    from distributed_tensorflow_example_amd.ops.conv import _bnb_fits

    shape = (2, 16, 4, 4)
    cl = torch.channels_last
    x = torch.zeros(shape).contiguous(memory_format=cl)
    stats = torch.zeros(4 * 16)
    plain = BwdSlot(x, stats)
    into = torch.zeros(shape, dtype=torch.bfloat16).contiguous(memory_format=cl)
    assert _bnb_fits(plain, None, shape)
    assert not _bnb_fits(plain, into, shape)           # a plain BN's gradient is this conv's alone
    assert not _bnb_fits(plain, None, (2, 16, 4, 2))   # another tensor's shape
    assert not _bnb_fits(BwdSlot(x, torch.zeros(8)), None, shape)
    res = BwdSlot(x, stats, torch.zeros(shape).contiguous(memory_format=cl))
    assert not _bnb_fits(res, None, shape)             # the residual branch's gradient must be folded in first
    assert _bnb_fits(res, into, shape)
    assert not _bnb_fits(res, into.float(), shape)
    assert not _bnb_fits(res, torch.zeros(shape, dtype=torch.bfloat16), shape)   # not channels_last
    assert not _bnb_fits(None, None, shape)


def test_fuse_bnb_prices_the_saved_passes(monkeypatch):
    from distributed_tensorflow_example_amd.ops import conv
    from distributed_tensorflow_example_amd.ops.bn import BwdSlot

    x = torch.zeros(128, 256, 14, 14)                  # 6.4M elements: one pass ~2.6 us at 5 TB/s
    key = ((128, 256, 14, 14), 64)
    plain, res = BwdSlot(x, None), BwdSlot(x, None, x)
    monkeypatch.setattr(conv, "_timings", {})
    assert conv._fuse_bnb(plain, "igemm", key, x)
    assert not conv._fuse_bnb(plain, "gemm_big", key, x)           # not timed: keep the chosen engine
    monkeypatch.setattr(conv, "_timings", {("dx",) + key: {"gemm_big": 0.0300, "igemm": 0.0320}})
    assert conv._fuse_bnb(plain, "gemm_big", key, x)               # 2.0 us behind < one 2.6 us pass
    monkeypatch.setattr(conv, "_timings", {("dx",) + key: {"gemm_big": 0.0300, "igemm": 0.0340}})
    assert not conv._fuse_bnb(plain, "gemm_big", key, x)           # 4 us behind > one pass
    assert conv._fuse_bnb(res, "gemm_big", key, x)                 # < two passes (residual form)


@pytest.mark.parametrize("bucket_mb", [0.001, 25.0])
def test_ddp_buckets_are_slices_of_one_flat_buffer(bucket_mb):
    from distributed_tensorflow_example_amd.models.mlp import MLP
    from distributed_tensorflow_example_amd.parallel.ddp import DistributedDataParallel
    from distributed_tensorflow_example_amd.parallel.world import World

    model = MLP(seed=0)
    ddp = DistributedDataParallel(model, World(), bucket_mb=bucket_mb)
    flat = ddp._flat
    for b in ddp.buckets:
        assert b.buf.untyped_storage().data_ptr() == flat.untyped_storage().data_ptr()
        assert (b.buf.data_ptr() - flat.data_ptr()) % 256 == 0          # 256-byte aligned slices
    for p in model.parameters():
        p.grad.fill_(1.0)
    ddp.zero_grad()
    assert all(float(p.grad.abs().sum()) == 0.0 for p in model.parameters())
    assert float(flat.abs().sum()) == 0.0
