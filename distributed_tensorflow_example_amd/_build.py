"""In-tree native build of the `_C` extension (HIP kernels + C++ runtime).

No hipify, no torch JIT cache: `.hip` sources are compiled by ``hipcc
--offload-arch=gfx950`` and host ``.cpp`` sources by ``g++`` against the
torch/ROCm headers; ninja drives the DAG (depfiles give incremental rebuilds)
and the result lands next to this file so it travels with the repo snapshot.

Usage: ``python -m distributed_tensorflow_example_amd._build [-j N] [--clean]``.
"""
from __future__ import annotations

import argparse
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(REPO, "csrc")
BUILD = os.path.join(REPO, "build", "native")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("DTF_OFFLOAD_ARCH", "gfx950")
EXT_NAME = "_C"


def ext_path() -> str:
    return os.path.join(PKG_DIR, EXT_NAME + sysconfig.get_config_var("EXT_SUFFIX"))


def sources():
    hip = sorted(glob.glob(os.path.join(CSRC, "**", "*.hip"), recursive=True))
    cpp = sorted(p for p in glob.glob(os.path.join(CSRC, "**", "*.cpp"), recursive=True)
                 if os.sep + "asan" + os.sep not in p)     # csrc/asan: the sanitizer build's own module
    return hip, cpp


def _torch_paths():
    import torch
    import torch.utils.cpp_extension as ce

    abi = int(bool(torch._C._GLIBCXX_USE_CXX11_ABI))
    return ce.include_paths(), ce.library_paths(), abi


def write_ninja() -> str:
    inc, libdirs, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    hip, cpp = sources()
    os.makedirs(BUILD, exist_ok=True)
    common_inc = [f"-I{CSRC}", f"-I{os.path.join(CSRC, 'kernels')}", f"-I{os.path.join(CSRC, 'runtime')}"]
    hip_flags = [
        f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
        "-fno-gpu-rdc", "-munsafe-fp-atomics", "-Wno-unused-result",
    ] + common_inc
    cxx_flags = [
        "-O2", "-fPIC", "-fvisibility=hidden", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_API_INCLUDE_EXTENSION_H",
        f"-DTORCH_EXTENSION_NAME={EXT_NAME}", "-Wno-deprecated-declarations", "-Wno-unused-result",
        f"-I{ROCM}/include", f"-I{py_inc}",
    ] + [f"-I{p}" for p in inc] + common_inc
    ldflags = ["-shared", f"-L{ROCM}/lib", "-lamdhip64", "-lrccl", "-lroctx64", "-lrocprofiler-sdk-roctx"]
    for d in libdirs:
        ldflags += [f"-L{d}", f"-Wl,-rpath,{d}"]
    ldflags += ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", "-lpthread"]

    lines = [
        "ninja_required_version = 1.5",
        f"hipcc = {ROCM}/bin/hipcc",
        "cxx = g++",
        "hipflags = " + " ".join(hip_flags),
        "cxxflags = " + " ".join(cxx_flags),
        "ldflags = " + " ".join(ldflags),
        "rule hip",
        "  command = $hipcc $hipflags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIPCC $in",
        "rule cxx",
        "  command = $cxx $cxxflags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $in",
        "rule link",
        "  command = $cxx $in $ldflags -o $out",
        "  description = LINK $out",
    ]
    objs = []
    for s in hip + cpp:
        rel = os.path.relpath(s, CSRC).replace(os.sep, "_")
        o = os.path.join(BUILD, rel + ".o")
        objs.append(o)
        lines.append(f"build {o}: {'hip' if s.endswith('.hip') else 'cxx'} {s}")
    lines.append(f"build {ext_path()}: link " + " ".join(objs))
    lines.append(f"default {ext_path()}")
    path = os.path.join(BUILD, "build.ninja")
    text = "\n".join(lines) + "\n"
    old = open(path).read() if os.path.exists(path) else None
    if old != text:
        with open(path, "w") as f:
            f.write(text)
    return path


def build(jobs: int | None = None, verbose: bool = False) -> str:
    """Build (incrementally) and return the path of the extension module."""
    write_ninja()
    if jobs is None:
        jobs = min(8, int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)))
    cmd = ["ninja", "-C", BUILD, f"-j{jobs}"]
    if verbose:
        cmd.append("-v")
    r = subprocess.run(cmd, capture_output=not verbose, text=True)
    if r.returncode != 0:
        out = (r.stdout or "") + (r.stderr or "")
        raise RuntimeError("native build failed:\n" + out[-20000:])
    return ext_path()


def is_stale() -> bool:
    p = ext_path()
    if not os.path.exists(p):
        return True
    t = os.path.getmtime(p)
    hip, cpp = sources()
    hdrs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    return any(os.path.getmtime(s) > t for s in hip + cpp + hdrs)


def clean():
    shutil.rmtree(BUILD, ignore_errors=True)
    if os.path.exists(ext_path()):
        os.remove(ext_path())


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args(argv)
    if a.clean:
        clean()
    print(build(a.j, a.v))


if __name__ == "__main__":
    sys.exit(main())
