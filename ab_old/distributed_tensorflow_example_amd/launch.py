"""Cluster launcher CLI (replaces run_lr2.sh / run.sh + the vendored shflags).

    python -m distributed_tensorflow_example_amd.launch filelist hdfs://nn/lr/train -R --min-size 1000
    python -m distributed_tensorflow_example_amd.launch local --ps 1 --workers 8 \
        examples/sparse_lr.py -- --features=1000000000 --train=... --test=...
    python -m distributed_tensorflow_example_amd.launch lr2 --run_mode test -j worker -i 0 -t <train> -T <test>
    python -m distributed_tensorflow_example_amd.launch lr2 --run_mode product -t <train> -T <test>

Reference behaviour:
* `get_file_list` (run_lr2.sh:39-47): `hadoop fs -ls -R path | awk 'NF>7 && $5>1000'`
  -> comma list of files bigger than 1000 B; run.sh:25-41 writes a newline
  list file and uploads it.  Here: gfile listing (local, fake-HDFS or the
  hadoop CLI backend), same size filter, comma or newline output,
  optional upload through gfile.
* `run_mode=test` (run_lr2.sh:60-71) runs one local lr2.py task with the
  given flags; `run_mode=product` submits the whole job through an external
  `tf_tool -c lr2.json` (not in the repo) with the product hyper-parameters
  (batch 500, 50 epochs, 1e9 features, 8 threads, lr 1, sampling 0.01/0.002).
  Here product mode launches the full cluster itself (`local`), one worker
  process per GPU.
* shflags' typed flags / short names (-j -i -t -T) / --help / validation are
  argparse; unknown flags are rejected like shflags' getopt.
`local` is also the failure detector: a task exiting non-zero (or being
killed) tears the whole job down with a report, instead of leaving the ps
blocked forever in join() (lr2.py:333-335).
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional

from .utils import gfile

PRODUCT_FLAGS = ["--batch_size=500", "--num_epochs=50", "--features=1000000000", "--thread_num=8",
                 "--learning_rate=1", "--trace_step_interval=10000", "--train_sampling_rate=0.01",
                 "--test_sampling_rate=0.002"]


# ----------------------------------------------------------------------- file lists
def list_files(path: str, recursive: bool = False, min_size: int = 0) -> List[str]:
    """Files under `path` (or matching a glob) with size > min_size, sorted."""
    out = []
    if any(c in path for c in "*?["):
        cands = gfile.Glob(path)
    elif gfile.IsDirectory(path):
        cands = [path.rstrip("/") + "/" + n for n in gfile.ListDirectory(path)]
    else:
        cands = [path]
    for c in sorted(cands):
        if gfile.IsDirectory(c):
            if recursive:
                out.extend(list_files(c, True, min_size))
            continue
        try:
            size = gfile.Stat(c).length
        except Exception:
            size = 0
        if size > min_size:
            out.append(c)
    return out


def cmd_filelist(a) -> int:
    files = list_files(a.path, a.recursive, a.min_size)
    text = (",".join(files) + ("," if files and a.trailing_comma else "")) if a.sep == "," else \
        "".join(f + "\n" for f in files)
    if a.out:
        with gfile.GFile(a.out, "w") as f:
            f.write(text)
    else:
        sys.stdout.write(text + ("\n" if a.sep == "," else ""))
    return 0


# ----------------------------------------------------------------------- local cluster
def free_ports(n: int, host: str = "127.0.0.1") -> List[int]:
    socks, ports = [], []
    for _ in range(n):
        s = socket.socket()
        s.bind((host, 0))
        socks.append(s)
        ports.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return ports


def make_cluster(num_ps: int, num_workers: int, host: str = "127.0.0.1", base_port: int = 0) -> Dict[str, List[str]]:
    n = num_ps + num_workers
    ports = list(range(base_port, base_port + n)) if base_port else free_ports(n, host)
    return {"ps": [f"{host}:{p}" for p in ports[:num_ps]],
            "worker": [f"{host}:{p}" for p in ports[num_ps:]]}


def run_local(script: str, num_ps: int, num_workers: int, script_args: List[str], log_dir: Optional[str] = None,
              gpus: Optional[List[int]] = None, cluster_flag: str = "--cluster_conf", timeout: float = 0,
              python: str = sys.executable, poll: float = 0.2) -> int:
    cluster = make_cluster(num_ps, num_workers)
    log_dir = log_dir or os.path.abspath("logs/launch")
    os.makedirs(log_dir, exist_ok=True)
    conf = os.path.join(log_dir, "cluster_conf.json")
    with open(conf, "w") as f:
        json.dump(cluster, f)
    procs: Dict[str, subprocess.Popen] = {}
    logs = {}
    env0 = dict(os.environ)
    env0.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    tasks = [("ps", i) for i in range(num_ps)] + [("worker", i) for i in range(num_workers)]
    for job, i in tasks:
        env = dict(env0)
        if job == "worker" and gpus:
            env["HIP_VISIBLE_DEVICES"] = str(gpus[i % len(gpus)])
        if job == "ps":
            env["HIP_VISIBLE_DEVICES"] = ""          # ps tasks are control-plane only
        name = f"{job}_{i}"
        logs[name] = open(os.path.join(log_dir, name + ".log"), "w")
        cmd = [python, script, f"--job_name={job}", f"--task_index={i}", f"{cluster_flag}={conf}"] + script_args
        procs[name] = subprocess.Popen(cmd, env=env, stdout=logs[name], stderr=subprocess.STDOUT,
                                       start_new_session=True)
    print(f"[launch] {len(tasks)} tasks, cluster {conf}, logs in {log_dir}", flush=True)
    t0 = time.time()
    rc = 0
    failed = None
    try:
        while True:
            states = {n: p.poll() for n, p in procs.items()}
            bad = [n for n, r in states.items() if r not in (None, 0)]
            if bad:
                failed = bad[0]
                rc = states[failed] if states[failed] > 0 else 1
                break
            if all(r is not None for r in states.values()):
                break
            if timeout and time.time() - t0 > timeout:
                failed, rc = "timeout", 124
                break
            time.sleep(poll)
    except KeyboardInterrupt:
        failed, rc = "interrupted", 130
    if failed:
        print(f"[launch] task {failed} failed (rc={rc}); stopping the job", flush=True)
        for n, p in procs.items():
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        deadline = time.time() + 10
        for p in procs.values():
            try:
                p.wait(max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
    for f in logs.values():
        f.close()
    for n, p in procs.items():
        print(f"[launch] {n}: rc={p.returncode}", flush=True)
    return rc


def cmd_local(a) -> int:
    gpus = [int(g) for g in a.gpus.split(",")] if a.gpus else None
    return run_local(a.script, a.ps, a.workers, a.script_args, a.log_dir, gpus, timeout=a.timeout)


# ----------------------------------------------------------------------- lr2 wrapper
def cmd_lr2(a) -> int:
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = a.script or os.path.join(here, "examples", "sparse_lr.py")
    train = ",".join(list_files(a.train, True, 1000))
    test = ",".join(list_files(a.test, True, 1000))
    print(f"train data: {train}\ntest data: {test}\nrun mode: {a.run_mode}\nload mode: {a.load_mode}", flush=True)
    if not train or not test:
        print("no input files (files must be > 1000 bytes)", file=sys.stderr)
        return 1
    if a.run_mode == "product":
        args = PRODUCT_FLAGS + [f"--train={train}", f"--test={test}", f"--mode={a.load_mode}"] + a.extra
        return run_local(script, a.num_ps, a.num_workers, args, a.log_dir,
                         [int(g) for g in a.gpus.split(",")] if a.gpus else None)
    cmd = [sys.executable, script, f"--job_name={a.job_name}", f"--task_index={a.task_index}",
           f"--train={train}", f"--test={test}", f"--mode={a.load_mode}", f"--learning_rate={a.learning_rate}",
           f"--num_epochs={a.num_epochs}", f"--batch_size={a.batch_size}", f"--features={a.features}"] + a.extra
    if a.cluster_conf:
        cmd.append(f"--cluster_conf={a.cluster_conf}")
    return subprocess.call(cmd)


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="dtf-launch", description=__doc__.split("\n\n")[0])
    sub = p.add_subparsers(dest="cmd", required=True)

    f = sub.add_parser("filelist", help="list input files (run.sh / get_file_list)")
    f.add_argument("path")
    f.add_argument("-R", "--recursive", action="store_true")
    f.add_argument("--min-size", type=int, default=0, help="keep files larger than this many bytes")
    f.add_argument("--sep", choices=[",", "newline"], default=",")
    f.add_argument("--trailing-comma", action="store_true", help="awk ORS=',' output (run_lr2.sh)")
    f.add_argument("--out", default="", help="write the list here (any gfile path) instead of stdout")
    f.set_defaults(fn=cmd_filelist)

    l = sub.add_parser("local", help="run a ps/worker job on this host")
    l.add_argument("script")
    l.add_argument("--ps", type=int, default=1)
    l.add_argument("--workers", type=int, default=1)
    l.add_argument("--gpus", default="", help="comma list of GPU ids for the workers (one each)")
    l.add_argument("--log-dir", default=None)
    l.add_argument("--timeout", type=float, default=0)
    l.add_argument("script_args", nargs=argparse.REMAINDER)
    l.set_defaults(fn=cmd_local)

    r = sub.add_parser("lr2", help="run_lr2.sh equivalent")
    r.add_argument("-j", "--job_name", default="ps")
    r.add_argument("-i", "--task_index", type=int, default=0)
    r.add_argument("-t", "--train", required=True)
    r.add_argument("-T", "--test", required=True)
    r.add_argument("--run_mode", choices=["product", "test"], default="product")
    r.add_argument("--load_mode", choices=["all", "queue"], default="queue")
    r.add_argument("--learning_rate", type=float, default=0.001)
    r.add_argument("--num_epochs", type=int, default=120)
    r.add_argument("--batch_size", type=int, default=500)
    r.add_argument("--features", type=int, default=4762348)
    r.add_argument("--output", default="", help="output root (checkpoints)")
    r.add_argument("--cluster_conf", default="")
    r.add_argument("--num_ps", type=int, default=1)
    r.add_argument("--num_workers", type=int, default=1)
    r.add_argument("--gpus", default="")
    r.add_argument("--log_dir", default=None)
    r.add_argument("--script", default="")
    r.add_argument("extra", nargs=argparse.REMAINDER)
    r.set_defaults(fn=cmd_lr2)
    return p


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    for k in ("script_args", "extra"):
        v = getattr(a, k, None)
        if v and v[0] == "--":
            setattr(a, k, v[1:])
    return a.fn(a)


if __name__ == "__main__":
    sys.exit(main())
