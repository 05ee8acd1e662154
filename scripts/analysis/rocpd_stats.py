#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 --kernel-trace database (rocpd sqlite, the default output format of
rocprofv3 in this image), split by launch geometry so the headline launch size can be read off on its own:
  rocpd_stats.py <run_results.db> [--csv OUT] [--top N] [--min-ms T]
Columns: kernel, grid (threads), workgroup, launches, avg / min / max / total duration (ms).  --min-ms keeps launches
of at least T ms (bench.py's 32768-frame launches share their grid with its 4096-frame small-batch launches)."""
import argparse
import csv
import sqlite3
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv", default=None)
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--min-ms", type=float, default=0.0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, grid_x, workgroup_x, count(*), avg(end - start), min(end - start), "
                     "max(end - start), sum(end - start) from kernels where end - start >= ? group by name, grid_x, workgroup_x "
                     "order by sum(end - start) desc", (int(a.min_ms * 1e6),)).fetchall()
    out = [["kernel", "grid", "workgroup", "launches", "avg_ms", "min_ms", "max_ms", "total_ms"]]
    for n, g, w, k, av, mn, mx, tot in rows[: a.top]:
        out.append([n, g, w, k, f"{av / 1e6:.4f}", f"{mn / 1e6:.4f}", f"{mx / 1e6:.4f}", f"{tot / 1e6:.2f}"])
    wr = csv.writer(open(a.csv, "w", newline="") if a.csv else sys.stdout)
    wr.writerows(out)


if __name__ == "__main__":
    main()
