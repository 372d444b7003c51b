"""Hogwild parameter store on the GPU: variables in rank 0's uncached device
memory, IPC-mapped into every rank, updated by csrc/kernels/hogwild.hip
(2-3 ranks sharing cuda:0, the IPC path the 8-GPU node uses over xGMI)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("nproc,locking,table", [(2, True, False), (3, True, False), (2, False, False),
                                                 (2, True, True), (3, True, True), (2, False, True)])
def test_hogwild_store_ipc_same_gpu(native, nproc, locking, table):
    """table: a row-sharded table (lr2.py's ps-held W) -- rows gathered from and
    scatter-SGD'd into the owners' IPC-mapped shards (csrc/kernels/hogwild.hip)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1",
           f"--master-port={port}", os.path.join(REPO, "scripts", "async_ps_selftest.py"), "--same-gpu"]
    if not locking:
        cmd.append("--no-locking")
    if table:
        cmd.append("--table")
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=100, env=env)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and line, (r.stdout + r.stderr)[-3000:]
    res = json.loads(line[-1])
    assert res["async_ps_selftest"] == "pass" and res["kind"] == "ipc", res
