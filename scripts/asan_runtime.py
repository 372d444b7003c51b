"""Build the C++ runtime with AddressSanitizer + UBSan (host code only) and
exercise every component under it.

    python scripts/asan_runtime.py            # ASan + UBSan: build build/asan/_rt_asan*.so, run the exercise
    python scripts/asan_runtime.py --tsan     # ThreadSanitizer build (build/tsan/), same exercise
    python scripts/asan_runtime.py --exercise # (internal) run inside the sanitized process

The runtime sources (csrc/runtime: TF bundle, tfevents/TFRecord writer, TCP
store, blocking queue, libsvm parser, CRC32C) are compiled by g++ with
-fsanitize=address,undefined into a separate module `_rt_asan` (the HIP
kernels are not part of it), loaded into a Python started with libasan
preloaded, and driven through concurrent and edge-case paths: multi-threaded
queue producers/consumers with close, a TCP store server with several client
threads, sliced/sharded bundle writes + merges + reads, TFRecord framing,
libsvm parsing of malformed lines.  Any ASan/UBSan report aborts the process
(halt_on_error), so exit code 0 == clean.
"""
from __future__ import annotations

import os
import subprocess
import sys
import sysconfig

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TSAN = "--tsan" in sys.argv
OUT = os.path.join(REPO, "build", "tsan" if TSAN else "asan")
RT = ["tf_bundle.cpp", "tfrecord.cpp", "tcp_store.cpp", "blocking_queue.cpp", "libsvm.cpp", "crc32c.cpp"]


def build() -> str:
    import torch
    import torch.utils.cpp_extension as ce

    os.makedirs(OUT, exist_ok=True)
    so = os.path.join(OUT, "_rt_asan" + sysconfig.get_config_var("EXT_SUFFIX"))
    srcs = [os.path.join(REPO, "csrc", "runtime", f) for f in RT] + [os.path.join(REPO, "csrc", "asan", "asan_module.cpp")]
    if os.path.exists(so) and all(os.path.getmtime(so) > os.path.getmtime(s) for s in srcs):
        return so
    abi = int(bool(torch._C._GLIBCXX_USE_CXX11_ABI))
    inc = ce.include_paths()
    libdirs = ce.library_paths()
    san = ["-fsanitize=thread", "-DDTF_TSAN"] if TSAN else ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"]
    flags = ["-O1", "-g", "-fPIC", "-std=c++17", "-fno-omit-frame-pointer"] + san + [ f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_API_INCLUDE_EXTENSION_H",
             "-DTORCH_EXTENSION_NAME=_rt_asan", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
             "-Wno-deprecated-declarations", f"-I{sysconfig.get_paths()['include']}", "-I/opt/rocm/include",
             f"-I{os.path.join(REPO, 'csrc', 'runtime')}"] + [f"-I{p}" for p in inc]
    objs = []
    for s in srcs:
        o = os.path.join(OUT, os.path.basename(s) + ".o")
        subprocess.run(["g++"] + flags + ["-c", s, "-o", o], check=True)
        objs.append(o)
    link = ["g++", "-shared", san[0], "-o", so] + objs
    for d in libdirs:
        link += [f"-L{d}", f"-Wl,-rpath,{d}"]
    link += ["-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lpthread"]
    subprocess.run(link, check=True)
    return so


def exercise():
    import tempfile
    import threading

    import numpy as np
    import torch  # noqa: F401

    sys.path.insert(0, OUT)
    import _rt_asan as R

    d = tempfile.mkdtemp()
    # --- TF bundle: plain + sliced entries, two shards, merge, reads
    prefix = os.path.join(d, "m.ckpt")
    full = np.arange(70, dtype=np.float32).reshape(7, 10)
    for shard, (a, n) in enumerate([(0, 4), (4, 3)]):
        w = R.BundleWriter(prefix, shard, 2)
        if shard == 0:
            w.add("b", 1, [3], np.ones(3, np.float32).view(np.uint8))
        w.add_slice("W", 1, [7, 10], [(a, n), (0, 10)], np.ascontiguousarray(full[a:a + n]).reshape(-1).view(np.uint8))
        w.finish()
    R.bundle_merge_shard_indexes(prefix, 2, True)
    idx = R.bundle_read_index(prefix)
    assert idx["W"]["slices"] == [[(0, 4), (0, 10)], [(4, 3), (0, 10)]], idx["W"]
    got = np.frombuffer(R.bundle_read_slice(prefix, "W", [(4, 3), (0, 10)], True), np.float32).reshape(3, 10)
    assert np.array_equal(got, full[4:])
    assert R.bundle_slice_key("a\x00b", [(5, 7)]) == b"\x00a\x00\xffb\x00\x01\x01\x01\x85\x87"
    # --- TFRecord framing
    recs = [b"", b"x" * 1000, bytes(range(256))]
    p = os.path.join(d, "r.tfrecord")
    R.write_records(p, recs)
    assert R.read_records(p) == recs
    # --- TCP store: server + concurrent clients
    srv = R.TCPStore("127.0.0.1", 0, True, 30.0)
    port = srv.port

    def client(i):
        c = R.TCPStore("127.0.0.1", port, False, 30.0)
        for j in range(50):
            c.set(f"k{i}_{j}", bytes([j % 256]) * 17)
            c.add("ctr", 1)
        assert c.get(f"k{i}_49") == bytes([49]) * 17
    ts = [threading.Thread(target=client, args=(i,)) for i in range(6)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert srv.add("ctr", 0) == 300
    # --- blocking queue: producers, consumers, close with waiters
    q = R.BlockingQueue(8)
    got_items = []

    def prod(i):
        for j in range(100):
            q.put((i, j))

    def cons():
        while True:
            try:
                it = q.get(5.0)
            except R.QueueClosedError:      # closed and drained
                return
            got_items.append(it)
    ps = [threading.Thread(target=prod, args=(i,)) for i in range(4)]
    cs = [threading.Thread(target=cons) for _ in range(3)]
    [t.start() for t in ps + cs]
    [t.join() for t in ps]
    q.close()
    [t.join() for t in cs]
    assert len(got_items) == 400, len(got_items)
    # --- libsvm parser incl. malformed tokens
    f = os.path.join(d, "a.svm")
    with open(f, "w") as fh:
        fh.write("1 3:0.5 7:1\n0 2:1.5\n1 bad 9:2\n\n0 1:1e-3 1000000:4\n")
    out = R.libsvm_parse_files([f], 2)
    assert out is not None
    st = R.LibsvmStream([f], 2, 2, 1.0, True, 4, 0)      # looping stream, 2 parser threads
    for _ in range(6):
        st.next(5.0)
    st.stop()
    print("asan runtime exercise: clean")


def main():
    if "--exercise" in sys.argv:
        return exercise()
    so = build()
    rt = "libtsan.so" if TSAN else "libasan.so"
    lib = subprocess.run(["gcc", f"-print-file-name={rt}"], capture_output=True, text=True).stdout.strip()
    cxx = subprocess.run(["gcc", "-print-file-name=libstdc++.so.6"], capture_output=True, text=True).stdout.strip()
    # libstdc++ right behind the sanitizer runtime: the interpreter itself does not
    # link it, and the __cxa_throw interceptor must resolve the real symbol
    env = dict(os.environ, LD_PRELOAD=f"{lib}:{cxx}",
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0:allocator_may_return_null=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               # races are reported for the runtime's own frames; the uninstrumented
               # interpreter / torch are not part of the exercise's verdict
               TSAN_OPTIONS="halt_on_error=1:report_signal_unsafe=0:ignore_noninstrumented_modules=1")
    args = ["--exercise"] + (["--tsan"] if TSAN else [])
    r = subprocess.run([sys.executable, os.path.abspath(__file__)] + args, env=env)
    print(f"sanitized module: {so}; exit {r.returncode}")
    sys.exit(r.returncode)


if __name__ == "__main__":
    main()
