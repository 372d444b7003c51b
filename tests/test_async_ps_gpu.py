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


@pytest.mark.parametrize("nproc,locking", [(2, True), (3, True), (2, False)])
def test_hogwild_store_ipc_same_gpu(native, nproc, locking):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1",
           f"--master-port={port}", os.path.join(REPO, "scripts", "async_ps_selftest.py"), "--same-gpu"]
    if not locking:
        cmd.append("--no-locking")
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=100, env=env)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and line, (r.stdout + r.stderr)[-3000:]
    res = json.loads(line[-1])
    assert res["async_ps_selftest"] == "pass" and res["kind"] == "ipc", res
