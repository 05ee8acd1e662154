#!/usr/bin/env python3
"""Latency of small gmm_score_host_ring calls (the drop-in's buffer sizes 1..64): wall time per call through the
C-ABI into page-locked frame-major tables, beside the scorer kernel's own time (HIP events), so the host/PCIe
overhead of a call is the difference.  Prints one JSON line per (type, frames per call).
usage: host_latency.py [--types diagonal-maximum,SIMD-diagonal-maximum] [--sizes 1,4,16,64] [--calls 300]"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--types", default="diagonal-maximum,SIMD-diagonal-maximum")
    ap.add_argument("--sizes", default="1,4,16,64")
    ap.add_argument("--calls", type=int, default=300)
    ap.add_argument("--nn", action="store_true", help="the hybrid-DNN scorer instead of the GMM types")
    a = ap.parse_args()
    import rasr_amd as ra
    ms = ra.synthetic_mixture_set(5000, 160, 39, seed=2024)
    R = max(64, max(int(v) for v in a.sizes.split(",")))
    frames = ra.synthetic_frames(R, 39, seed=7)
    if a.nn:  # the hybrid-DNN scorer's host call (bench.py NN_DIMS), frame-major into a page-locked table
        from rasr_amd import nn
        dims = [429] + [2048] * 6 + [5000]
        sc = nn.NnScorer(nn.synthetic_network(dims, "sigmoid", seed=3), max_frames=R)
        x = ra.pinned_empty((R, dims[0]))
        x[:] = ra.synthetic_frames(R, dims[0], seed=9)
        out = ra.pinned_empty((R, dims[-1]))
        for n in (int(v) for v in a.sizes.split(",")):
            for _ in range(10):
                sc.score_host(x, out=out, n_frames=n, frame_major=True)
            sc.set_timing(True)
            sc.kernel_time(reset=True)
            wall = []
            for _ in range(a.calls // 3):
                t0 = time.perf_counter()
                sc.score_host(x, out=out, n_frames=n, frame_major=True)
                wall.append(time.perf_counter() - t0)
            kms, launches = sc.kernel_time(reset=True)
            sc.set_timing(False)
            med = statistics.median(wall) * 1e6
            print(json.dumps({"type": "hybrid-dnn", "frames_per_call": n, "call_us_median": round(med, 1),
                              "layers_us": round(kms * 1e3 / max(launches, 1), 1),
                              "frames_per_s": round(n / (med * 1e-6), 1)}), flush=True)
        return
    for kind in a.types.split(","):
        sc = ra.Scorer(ms, kind, max_frames=R)
        ring = ra.pinned_empty((R, 39))
        ring[:] = frames
        out = ra.pinned_empty((R, sc.n_mixtures()))
        for n in (int(x) for x in a.sizes.split(",")):
            for _ in range(20):
                sc.score_host_ring(ring, 0, n, out, frame_major=True)
            sc.set_timing(True)
            sc.kernel_time(reset=True)
            wall = []
            for i in range(a.calls):
                t0 = time.perf_counter()
                sc.score_host_ring(ring, (i * n) % R, n, out, frame_major=True)
                wall.append(time.perf_counter() - t0)
            kms, launches = sc.kernel_time(reset=True)
            sc.set_timing(False)
            med = statistics.median(wall) * 1e6
            kern = kms * 1e3 / max(launches, 1)
            print(json.dumps({"type": kind, "frames_per_call": n, "call_us_median": round(med, 1),
                              "call_us_min": round(min(wall) * 1e6, 1), "kernel_us": round(kern, 1),
                              "overhead_us": round(med - kern, 1), "frames_per_s": round(n / (med * 1e-6), 1)}),
                  flush=True)
        sc.close()


if __name__ == "__main__":
    main()
