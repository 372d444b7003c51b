"""Loader for the in-tree native extension `_C` (HIP kernels + C++ runtime).

`torch` is imported first so that torch's HIP runtime and RCCL are the ones the
extension binds to (same SONAMEs).  If the module is missing -- or STALE: built
from other sources than this tree's, judged by the source hash embedded in the
binary (`_build.src_hash`, also `_C.SRC_HASH`) -- it is (re)built in-tree
(ninja + hipcc for gfx950) before the import; a file lock keeps concurrent
ranks from building at once.  A stale binary never loads silently:
`DTF_NATIVE_STALE=error` turns staleness into an ImportError instead of a
rebuild.  On a GPU box a missing/broken extension is a hard error -- ops never
fall back silently to eager PyTorch there.
"""
from __future__ import annotations

import fcntl
import importlib
import os
import threading

_lock = threading.Lock()
_C = None
_err: Exception | None = None


def load(build_if_missing: bool = True):
    """Return the `_C` module, building it in-tree if it is absent."""
    global _C, _err
    if _C is not None:
        return _C
    with _lock:
        if _C is not None:
            return _C
        import torch  # noqa: F401  (bind to torch's libamdhip64 / librccl)

        from . import _build

        path = _build.ext_path()
        force = os.environ.get("DTF_FORCE_REBUILD", "0") == "1"
        if force or _build.is_stale():
            why = "missing" if not os.path.exists(path) else (
                "forced" if force else f"stale (built from {_build.built_hash()}, tree is {_build.src_hash()})")
            if not build_if_missing:
                raise ImportError(f"native extension {why}: {path}")
            if os.environ.get("DTF_NATIVE_STALE") == "error" and os.path.exists(path) and not force:
                raise ImportError(f"native extension {why}: {path} (DTF_NATIVE_STALE=error)")
            os.makedirs(os.path.dirname(_build.BUILD), exist_ok=True)
            lock_path = os.path.join(os.path.dirname(_build.BUILD), ".native_build.lock")
            with open(lock_path, "w") as lf:
                fcntl.flock(lf, fcntl.LOCK_EX)
                try:
                    if force or _build.is_stale():
                        print(f"[native] building _C: {why}", flush=True)
                        _build.build()
                finally:
                    fcntl.flock(lf, fcntl.LOCK_UN)
        try:
            _C = importlib.import_module(__package__ + "._C")
        except Exception as e:  # pragma: no cover - surfaced to caller
            _err = e
            raise
        return _C


def available() -> bool:
    try:
        load()
        return True
    except Exception:
        return False


def src_hash() -> str:
    """Source hash of the loaded `_C` (what the bench line reports)."""
    return str(getattr(load(), "SRC_HASH", "unknown"))


def native_path() -> str:
    from . import _build

    return _build.ext_path()
