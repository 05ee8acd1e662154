"""Per-layer kernel durations of bench.py --mode nn from a rocprofv3 --kernel-trace CSV: dispatches of
the NN GEMM grouped by grid size (one grid size per layer shape)."""
import csv
import glob
import sys
from collections import defaultdict

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
by = defaultdict(list)
for r in rows:
    if "nnGemm" in r["Kernel_Name"]:
        by[(r["Kernel_Name"].split("(")[0], r.get("Grid_Size_X", r.get("Grid_Size", "?")))].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    v = sorted(v)
    print(k, "n", len(v), "median us", round(v[len(v) // 2], 1), "min", round(v[0], 1))
