#!/usr/bin/env python3
"""Per-kernel, per-grid dispatch statistics from a rocprofv3 --kernel-trace database (rocpd SQLite, the ROCm 7
default output): rocprofv3's own --stats table averages every launch size of a kernel together, while bench.py's
roofline is per launch size, so the grid size (the launch's frame tiles x chunks) is kept as a key.

usage: rocpd_stats.py <run_results.db> [--csv out.csv] [--top N]
Columns: kernel, grid_x, workgroup_x, vgpr, lds_bytes, calls, total_us, avg_us, min_us, max_us, percent.
"""
import argparse
import csv
import sqlite3
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute(
        "select name, grid_x, workgroup_x, max(vgpr_count + accum_vgpr_count), max(lds_size), count(*), "
        "sum(duration), avg(duration), min(duration), max(duration) from kernels "
        "group by name, grid_x, workgroup_x order by sum(duration) desc").fetchall()
    total = sum(r[6] for r in rows) or 1
    out = []
    for name, gx, wx, vgpr, lds, n, tot, avg, mn, mx in rows:
        out.append({"kernel": name.split("(")[0], "grid_x": gx, "workgroup_x": wx, "vgpr": vgpr, "lds_bytes": lds,
                    "calls": n, "total_us": round(tot / 1e3, 3), "avg_us": round(avg / 1e3, 3),
                    "min_us": round(mn / 1e3, 3), "max_us": round(mx / 1e3, 3),
                    "percent": round(100.0 * tot / total, 3)})
    w = csv.DictWriter(open(a.csv, "w") if a.csv else sys.stdout, fieldnames=list(out[0].keys()))
    w.writeheader()
    for r in out[: a.top] if not a.csv else out:
        w.writerow(r)


if __name__ == "__main__":
    main()
