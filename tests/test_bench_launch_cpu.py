"""bench.py's launch shapes without a GPU: `--gpus N` as one plain process
starts its own N rank processes (the reference's hand-launched tasks,
README.md:11-16), forwards rank 0's single JSON line and returns the worst
rank exit code; the lazy, bounded RCCL bring-up agrees on failure across
ranks (World.ensure_comm)."""
import json
import os
import subprocess
import sys
import textwrap
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

_RANK_SCRIPT = textwrap.dedent("""
    import json, os, sys, time
    r, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert os.environ["LOCAL_RANK"] == str(r) and os.environ["MASTER_ADDR"] == "127.0.0.1"
    assert int(os.environ["MASTER_PORT"]) > 0 and os.environ["DTF_BENCH_SELF_LAUNCHED"] == "1"
    mode = sys.argv[1]
    print(f"rank {r} chatter")               # non-JSON stdout of every rank
    if mode == "hang" and r == 2:
        time.sleep(600)
    if mode in ("fail", "hang") and r == 1:
        sys.exit(7)
    if r == 0:
        print(json.dumps({"n_gpus": n, "args": sys.argv[1:]}))
""")


def _launch(tmp_path, mode, n, grace=60.0):
    script = tmp_path / "rank.py"
    script.write_text(_RANK_SCRIPT)
    code = textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {REPO!r})
        import os
        for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
            os.environ.pop(k, None)
        import bench
        sys.exit(bench.self_launch([{mode!r}, "--gpus", "{n}"], {n}, grace_s={grace}, script={str(script)!r}))
    """)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR")}
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
    return p, time.monotonic() - t0


def test_self_launch_forwards_rank0_line(tmp_path):
    p, _ = _launch(tmp_path, "ok", 4)
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 2, p.stdout          # rank 0's chatter + its one JSON line
    assert json.loads(lines[-1]) == {"n_gpus": 4, "args": ["ok", "--gpus", "4"]}
    assert "rank 3 chatter" in p.stderr       # other ranks' stdout goes to stderr


def test_self_launch_returns_failing_rank_code(tmp_path):
    p, _ = _launch(tmp_path, "fail", 3)
    assert p.returncode == 7, p.stderr


def test_self_launch_terminates_hung_rank_after_failure(tmp_path):
    p, dt = _launch(tmp_path, "hang", 3, grace=2.0)
    assert p.returncode == 7, p.stderr
    assert dt < 60, dt


def _ensure_comm_worker(rank, world, port, fault, q):
    import datetime

    import torch.distributed as dist

    from distributed_tensorflow_example_amd.parallel import world as W

    if fault:
        os.environ["DTF_FAULT_RCCL_INIT"] = "1"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))
    w = W.World(rank=rank, world_size=world, backend="gloo", pg_initialized=True)
    out = []
    for _ in range(2):
        try:
            out.append(("ok", w.ensure_comm()))
        except RuntimeError as e:
            out.append(("err", str(e)))
    # the data plane still works over gloo afterwards
    import torch
    t = torch.ones(3) * (rank + 1)
    w.all_reduce(t)
    out.append(("sum", float(t[0])))
    q.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.parametrize("fault", [False, True])
def test_ensure_comm_agrees_across_ranks(fault):
    import multiprocessing as mp
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_ensure_comm_worker, args=(r, 2, port, fault, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for r in range(2):
        out = res[r]
        if fault:
            assert out[0][0] == "err" and "fault injected" in out[0][1]
            assert out[1] == out[0]                    # recorded: no second attempt
        else:
            assert out[0] == ("ok", None) and out[1] == ("ok", None)   # gloo world: no RCCL data plane
        assert out[2] == ("sum", 3.0)
