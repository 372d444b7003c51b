"""The IPC collectives (csrc/kernels/ipc_coll.hip, csrc/comm/ipc_coll.cpp) --
World's RCCL-free GPU data plane -- with 2, 3 and 4 ranks sharing cuda:0:
every collective against an exact rank-order expectation, chunking past a
small slot capacity, a captured hipGraph replayed with new inputs, and a
skipped collective that must time out on the waiting ranks and raise
(scripts/ipc_coll_selftest.py)."""
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


def _run(nproc, *args, env_extra=None, timeout=200):
    cmd = [sys.executable, "-m", "torch.distributed.run", f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1",
           f"--master-port={_port()}", os.path.join(REPO, "scripts", "ipc_coll_selftest.py")] + list(args)
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="2", DTF_DATA_PLANE="ipc", DTF_IPC_SLOT_MB="1",
               DTF_IPC_TIMEOUT_S="20")
    env.update(env_extra or {})
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    out = r.stdout + r.stderr
    assert lines, out[-3000:]
    return r.returncode, json.loads(lines[-1]), out


@pytest.mark.parametrize("nproc", [2, 3, 4])
def test_ipc_collectives_same_gpu(native, nproc):
    rc, res, out = _run(nproc)
    assert rc == 0 and res["ipc_coll_selftest"] == "pass", (res, out[-2000:])
    assert not res["rccl_comm"]          # the whole run without an RCCL communicator


def test_ipc_collective_timeout_raises(native):
    rc, res, out = _run(2, "--fault", env_extra={"DTF_IPC_TIMEOUT_S": "2"})
    assert rc == 0 and res["ipc_coll_fault"] == "pass", (res, out[-2000:])
