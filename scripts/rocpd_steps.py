"""Per-step kernel summary of the last N training steps in a rocprofv3
--kernel-trace database, cut at the step boundaries marked by a kernel that
runs once per step (default: the fused optimizer, multi_tensor_apply).

    python scripts/rocpd_steps.py <results.db> --steps N [--marker NAME] [--top K] [--context PAT]

--context PAT: also print, for the last step, each kernel whose name contains
PAT with the two kernels before and after it (which op issued a glue kernel).
"""
import argparse
import sqlite3
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--steps", type=int, required=True)
ap.add_argument("--marker", default="multi_tensor_apply")
ap.add_argument("--top", type=int, default=40)
ap.add_argument("--context", default=None)
a = ap.parse_args()
c = sqlite3.connect(a.db)
rows = c.execute("select name, start, end from kernels order by start").fetchall()
ends = [e for n, s, e in rows if a.marker in n]
if len(ends) <= a.steps:
    raise SystemExit(f"only {len(ends)} '{a.marker}' dispatches")
lo, hi = ends[-a.steps - 1], ends[-1]
tot, cnt = defaultdict(float), defaultdict(int)
for n, s, e in rows:
    if s > lo and e <= hi:
        tot[n] += (e - s) / 1e3
        cnt[n] += 1
busy = sum(tot.values())
print(f"window {(hi - lo) / 1e6:.2f} ms, kernel-busy {busy / 1e3:.2f} ms, per step {busy / a.steps:.1f} us")
print("  us/step calls/step   avg us    pct  kernel")
for n, t in sorted(tot.items(), key=lambda kv: -kv[1])[:a.top]:
    print(f"{t / a.steps:9.1f} {cnt[n] / a.steps:10.1f} {t / cnt[n]:8.1f} {100 * t / busy:6.2f}  {n[:150]}")
if a.context:
    last = [(n, s, e) for n, s, e in rows if s > ends[-2] and e <= hi]
    print(f"--- kernels around '{a.context}' in the last step")
    for i, (n, s, e) in enumerate(last):
        if a.context in n:
            for j in range(max(0, i - 2), min(len(last), i + 3)):
                mark = ">>" if j == i else "  "
                print(f"{mark} {(last[j][2] - last[j][1]) / 1e3:7.1f} us  {last[j][0][:110]}")
            print()
