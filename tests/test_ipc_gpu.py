"""One-shot IPC all-reduce (fused into the MLP SGD apply) with 2 and 3 ranks
sharing cuda:0: exercises IPC mapping, epoch flags and double-buffered
gradient slots on a 1-GPU box (the 8-GPU xGMI run uses the same code)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("mode", ["ipc-fused", "ipc-apply"])
@pytest.mark.parametrize("nproc", [2, 3])
def test_ipc_allreduce_same_gpu(native, nproc, mode):
    cmd = [sys.executable, "-m", "torch.distributed.run", f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1",
           f"--master-port={_port()}", os.path.join(REPO, "scripts", "ipc_selftest.py"), "--same-gpu",
           "--steps=12"]
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="2", DTF_IPC_MODE=mode)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    out = r.stdout + r.stderr
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and line, "\n".join(line) + "\n" + out[:1500] + "\n...\n" + out[-1500:]
    res = json.loads(line[-1])
    assert res["ipc_selftest"] == "pass", res
