"""Summarise a rocprofv3 kernel trace: per-kernel totals after a warm-up cut.

usage: prof_summary.py run_kernel_trace.csv --steps N [--after-last SUBSTR] [--top K]
Kernels that start before the end of the last kernel whose name contains
SUBSTR (e.g. MIOpen's solver-search 'naive_conv') are dropped, so a profile
of a run that benchmarks convolution solvers in its warm-up reports the
steady state only.
"""
import argparse
import csv
import re
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--steps", type=int, required=True, help="steps in the kept window (per-step averages)")
ap.add_argument("--after-last", default="")
ap.add_argument("--top", type=int, default=30)
ap.add_argument("--tail-ms", type=float, default=0.0,
                help="keep only kernels starting in the last T ms of the trace (a run's timed steps at its end)")
a = ap.parse_args()
rows = list(csv.DictReader(open(a.trace)))
cut = 0
if a.after_last:
    ends = [int(r["End_Timestamp"]) for r in rows if a.after_last in r["Kernel_Name"]]
    cut = max(ends) if ends else 0
if a.tail_ms > 0 and rows:
    cut = max(cut, max(int(r["End_Timestamp"]) for r in rows) - int(a.tail_ms * 1e6))
tot, cnt = defaultdict(float), defaultdict(int)
t0, t1 = None, 0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < cut:
        continue
    n = re.sub(r"\(.*", "", r["Kernel_Name"])[:110]
    tot[n] += e - s
    cnt[n] += 1
    t0 = s if t0 is None else min(t0, s)
    t1 = max(t1, e)
busy = sum(tot.values())
print(f"window {(t1 - (t0 or 0)) / 1e6:.2f} ms, kernel-busy {busy / 1e6:.2f} ms, per step {busy / a.steps / 1e3:.1f} us")
print(f"{'us/step':>9} {'calls/step':>10} {'avg us':>8}  kernel")
for n, v in sorted(tot.items(), key=lambda x: -x[1])[:a.top]:
    print(f"{v / a.steps / 1e3:9.1f} {cnt[n] / a.steps:10.1f} {v / cnt[n] / 1e3:8.1f}  {n}")
