"""Build hygiene of the in-tree `_C`: a binary built from other sources than
the tree's is detected by content (the source hash embedded in the .so) and
rebuilt by `_native.load()` before it is imported -- a stale binary never runs
silently."""
import os
import shutil

import pytest

from distributed_tensorflow_example_amd import _build, _native


def test_built_extension_carries_the_tree_hash():
    C = _native.load()
    assert C.SRC_HASH == _build.src_hash() == _build.built_hash()
    assert not _build.is_stale()


def test_touching_a_kernel_source_changes_the_hash(tmp_path, monkeypatch):
    csrc = tmp_path / "csrc"
    shutil.copytree(_build.CSRC, csrc)
    monkeypatch.setattr(_build, "CSRC", str(csrc))
    h0 = _build.src_hash()
    hip = csrc / "kernels" / "random.hip"
    hip.write_text(hip.read_text() + "\n// touched\n")
    h1 = _build.src_hash()
    assert h1 != h0
    # a header counts too
    hdr = csrc / "kernels" / "common.h"
    hdr.write_text(hdr.read_text() + "\n")
    assert _build.src_hash() not in (h0, h1)
    # mtimes alone do not: copy back the bytes with new timestamps
    shutil.copy(os.path.join(str(_build.REPO), "csrc", "kernels", "random.hip"), hip)
    shutil.copy(os.path.join(str(_build.REPO), "csrc", "kernels", "common.h"), hdr)
    os.utime(hip)
    assert _build.src_hash() == h0


def test_built_hash_reads_the_marker_without_importing(tmp_path):
    so = tmp_path / "fake.so"
    so.write_bytes(b"\x7fELF" + b"\0" * 100 + _build.HASH_MARK + b"0123456789abcdef" + b"\0" * 50)
    assert _build.built_hash(str(so)) == "0123456789abcdef"
    so.write_bytes(b"no marker here")
    assert _build.built_hash(str(so)) is None
    assert _build.built_hash(str(tmp_path / "missing.so")) is None


def test_load_rebuilds_a_stale_extension(monkeypatch):
    calls = []
    monkeypatch.setattr(_native, "_C", None)
    stale = iter([True, True, False])     # before the lock, under the lock, (after)
    monkeypatch.setattr(_build, "is_stale", lambda: next(stale, False))
    monkeypatch.setattr(_build, "build", lambda *a, **k: calls.append("build") or _build.ext_path())
    C = _native.load()
    assert calls == ["build"] and C.ARCH == "gfx950"


def test_stale_extension_can_be_made_an_error(monkeypatch):
    monkeypatch.setattr(_native, "_C", None)
    monkeypatch.setattr(_build, "is_stale", lambda: True)
    monkeypatch.setattr(_build, "build", lambda *a, **k: pytest.fail("must not build"))
    monkeypatch.setenv("DTF_NATIVE_STALE", "error")
    with pytest.raises(ImportError, match="stale"):
        _native.load()
