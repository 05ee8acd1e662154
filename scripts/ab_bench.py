#!/usr/bin/env python3
"""A/B timing of library variants (scripts/build_variants.sh) on one GPU.

Each variant runs in its own subprocess (RASR_GMM_LIB=<so>); rounds are interleaved
(v1 v2 ... v1 v2 ...) and the median / min kernel time per variant is reported.
usage: ab_bench.py --mode fp32|simd|sum|bint|simds|fp32s|pint|pfloat --rounds 3 lib1.so lib2.so[:split16|:split32|:fullkeys] ...
(":split16" / ":split32" run that library with GMM_FLAG_SPLIT_TILE16 / _TILE32, ":fullkeys" with GMM_FLAG_FULL_KEYS;
"@N" at the end sets RASR_GMM_TARGET_BLOCKS=N for that arm, e.g. lib.so@4096 or lib.so:fullkeys@4096;
bint = batch-diagonal-maximum-int, scores only; simds = SIMD-diagonal-maximum without best densities; fp32s =
diagonal-maximum without best densities; pint / pfloat = preselection-batch-int / -float)
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import os, sys, json, time
sys.path.insert(0, os.environ["ROOT"])
import torch, rasr_amd as ra
mode = os.environ["MODE"]; F = int(os.environ["FRAMES"])
kind = {"fp32": "diagonal-maximum", "simd": "SIMD-diagonal-maximum", "sum": "diagonal-sum",
        "bint": "batch-diagonal-maximum-int", "simds": "SIMD-diagonal-maximum", "fp32s": "diagonal-maximum",
        "pint": "preselection-batch-int", "pfloat": "preselection-batch-float"}[mode]
D = int(os.environ.get("DIM", "39"))
ms = ra.synthetic_mixture_set(5000, 160, D, seed=2024)
opt = os.environ.get("OPT", "")
sc = ra.Scorer(ms, kind, max_frames=F, split_tile16=opt == "split16", split_tile32=opt == "split32",
               full_keys=opt == "fullkeys")
fr = torch.from_numpy(ra.synthetic_frames(F, D, seed=5)).cuda()
out = torch.empty((5000, F), dtype=torch.float32, device="cuda")
best = (torch.zeros((5000, F), dtype=torch.int32, device="cuda")
        if mode not in ("bint", "simds", "fp32s", "pint", "pfloat") else None)
for _ in range(3): sc.score_device(fr, out, best)
torch.cuda.synchronize(); sc.set_timing(True)
for _ in range(int(os.environ["STEPS"])): sc.score_device(fr, out, best)
ms_, n = sc.kernel_time()
w = torch.arange(1, F + 1, device="cuda", dtype=torch.int64) * 2654435761 % 1000003
key = out.view(torch.int32).long() + (7 * best.long() if best is not None else 0)
h = int((key * w).sum(dim=1).remainder(2**61 - 1).sum())
print(json.dumps({"kernel_ms": ms_ / n, "checksum": float(out[:, :64].double().sum()), "hash": h}))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="fp32")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--frames", type=int, default=0)
    ap.add_argument("--dim", type=int, default=39)
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    frames = a.frames or (8192 if a.mode == "fp32" else 32768)
    res = {lib: [] for lib in a.libs}
    sums = {}
    for _ in range(a.rounds):
        for lib in a.libs:
            spec, _, blocks = lib.partition("@")
            path, _, opt = spec.partition(":")
            env = dict(os.environ, RASR_GMM_LIB=os.path.abspath(path), ROOT=ROOT, MODE=a.mode, FRAMES=str(frames),
                       STEPS=str(a.steps), DIM=str(a.dim), OPT=opt)
            if blocks:
                env["RASR_GMM_TARGET_BLOCKS"] = blocks
            p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(lib, "FAILED", p.stderr[-2000:])
                sys.exit(p.returncode)
            r = json.loads(p.stdout.strip().splitlines()[-1])
            res[lib].append(r["kernel_ms"])
            sums[lib] = (r["checksum"], r["hash"])
    for lib, v in res.items():
        fps = frames / (statistics.median(v) * 1e-3)
        print(f"{os.path.basename(lib):40s} median {statistics.median(v):.4f} ms  min {min(v):.4f}  "
              f"{fps / 1e6:.3f} Mframes/s  checksum {sums[lib][0]:.6f} hash {sums[lib][1]}")


if __name__ == "__main__":
    main()
