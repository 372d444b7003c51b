"""Per-step kernel summary of the last N training steps in a rocprofv3
--kernel-trace database, cut at the step boundaries marked by a kernel that
runs once per step (default: the fused optimizer, multi_tensor_apply).

    python scripts/rocpd_steps.py <results.db> --steps N [--marker NAME] [--top K]
"""
import argparse
import sqlite3
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--steps", type=int, required=True)
ap.add_argument("--marker", default="multi_tensor_apply")
ap.add_argument("--top", type=int, default=40)
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
