#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (scripts/profile_pmc.sh) for one kernel.

usage: pmc_summary.py <dir with p*/run_counter_collection.csv> <kernel substring> [--json out.json]
                      [--algo-bytes N]

Per-dispatch averages of every counter, the effective clock (GRBM_GUI_ACTIVE is
summed over the 8 XCDs, MI355X_MICROARCH.md 'DVFS give-back'), and HBM traffic
per launch with the gfx950 correction (FETCH_SIZE reads half of a wide streaming
read: doubled; WRITE_SIZE exact; both in KiB), MI355X_MICROARCH.md section HBM.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("kernel")
    ap.add_argument("--json")
    ap.add_argument("--frames-per-launch", type=int, default=32768,
                    help="frames per scorer call of the profiled run (bench.py uses the summary only if it matches)")
    args = ap.parse_args()
    vals = defaultdict(list)
    dur = []
    for f in sorted(glob.glob(os.path.join(args.dir, "p*", "*counter_collection.csv"))):
        seen = set()
        for row in csv.DictReader(open(f)):
            if args.kernel not in row["Kernel_Name"]:
                continue
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
            key = row["Dispatch_Id"]
            if key not in seen:
                seen.add(key)
                dur.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    t = sum(dur) / len(dur) if dur else float("nan")
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from rasr_amd import _capi
    kernel_id = _capi.load_library().gmm_kernel_id().decode()
    out = {"kernel": args.kernel, "dispatches_per_pass": len(vals.get("SQ_WAVES", [])), "avg_duration_s": t,
           "kernel_id": kernel_id, "frames_per_launch": args.frames_per_launch, "counters": avg}
    if "GRBM_GUI_ACTIVE" in avg:
        out["effective_clock_ghz"] = avg["GRBM_GUI_ACTIVE"] / 8 / t / 1e9
    if "FETCH_SIZE" in avg or "WRITE_SIZE" in avg:
        fetch = 2 * avg.get("FETCH_SIZE", 0) * 1024
        write = avg.get("WRITE_SIZE", 0) * 1024
        out["hbm_fetch_bytes_per_launch_corrected"] = fetch
        out["hbm_write_bytes_per_launch"] = write
        out["hbm_bytes_per_launch"] = fetch + write
        out["hbm_gbs"] = (fetch + write) / t / 1e9
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
        # busy cycles summed over all SIMDs (1024) vs elapsed cycles
        out["mfma_busy_frac"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (avg["GRBM_GUI_ACTIVE"] / 8 * 1024)
    if "TCC_HIT_sum" in avg:
        out["l2_hit_rate"] = avg["TCC_HIT_sum"] / max(1.0, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    print(json.dumps(out, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
