#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 --kernel-trace database (rocpd SQLite, the ROCm 7 default output):
kernel, grid, workgroup, launches, avg/min/max/total ms -- the columns of profiles/r05/*/kernel_stats.csv.
usage: rocpd_stats.py <run_results.db> [--min-ms X] > kernel_stats.csv"""
import argparse
import csv
import sqlite3
import sys
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--min-ms", type=float, default=0.0, help="only dispatches at least this long (e.g. 3 for 32768-frame launches)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    names = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    groups = defaultdict(list)
    for kid, start, end, gx, wx in c.execute(
            "select kernel_id, start, end, grid_size_x, workgroup_size_x from rocpd_kernel_dispatch"):
        ms = (end - start) * 1e-6
        if ms >= a.min_ms:
            groups[(names.get(kid, str(kid)), gx, wx)].append(ms)
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "grid", "workgroup", "launches", "avg_ms", "min_ms", "max_ms", "total_ms"])
    for (name, gx, wx), v in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, gx, wx, len(v), f"{sum(v) / len(v):.4f}", f"{min(v):.4f}", f"{max(v):.4f}", f"{sum(v):.2f}"])


if __name__ == "__main__":
    main()
