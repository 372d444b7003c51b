"""Per-kernel summary (CSV) of a rocprofv3 --kernel-trace database (rocpd SQLite).

    python scripts/rocpd_summary.py gpurun_out/<dir>/<name>_results.db [out.csv] [--after NAME]

--after NAME keeps only kernels that start after the last dispatch whose name
contains NAME ends (e.g. the spin marker bench_models.py --trace-marker puts
right before its timed loop: the steady state without initialisation).

Columns: kernel name, calls, total_us, avg_us, pct, vgpr, sgpr, lds, scratch, grid.
"""
import csv
import sqlite3
import sys


def main():
    args = sys.argv[1:]
    if not args or args[0] in ("-h", "--help"):
        raise SystemExit(__doc__)
    after = None
    if "--after" in args:
        i = args.index("--after")
        after = args[i + 1]
        args = args[:i] + args[i + 2:]
    db = args[0]
    out = args[1] if len(args) > 1 else None
    # read-only: a mistyped path must not create an empty database
    c = sqlite3.connect(f"file:{db}?mode=ro", uri=True)
    where = ""
    if after:
        t = c.execute("select max(end) from kernels where name like ?", (f"%{after}%",)).fetchone()[0]
        if t is None:
            raise SystemExit(f"no kernel matching {after!r}")
        where = f"where start > {int(t)}"
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), max(vgpr_count), max(sgpr_count), max(lds_size), "
        f"max(scratch_size), max(grid_x * grid_y * grid_z) from kernels {where} group by name order by sum(duration) desc"
    ).fetchall()
    tot = sum(r[2] for r in rows) or 1
    table = [["kernel", "calls", "total_us", "avg_us", "pct", "vgpr", "sgpr", "lds_bytes", "scratch", "grid_threads"]]
    for name, n, s, a, v, sg, l, sc, gr in rows:
        table.append([name[:160], n, round(s / 1e3, 2), round(a / 1e3, 3), round(100.0 * s / tot, 2), v, sg, l, sc, gr])
    f = open(out, "w", newline="") if out else sys.stdout
    csv.writer(f).writerows(table)


if __name__ == "__main__":
    main()
