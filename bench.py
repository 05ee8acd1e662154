#!/usr/bin/env python3
"""bench.py -- frames/s of the MI355X diagonal-GMM scorer (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 800k-density triphone diag-GMM, 39-dim,
5000 mixtures x 160 densities, pooled covariance, synthetic model and frames
(SURVEY.md 8(d)); one step = scoring one batch of F frames per GPU against every
mixture (scores + best densities written to HBM), inputs resident in HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--mode fp32|simd] [--frames F]

N > 1 is launched by torch.distributed.run: every rank scores its own frame
shard against a replica of the model (no collective on the data path,
"scaling": "weak"); a barrier + synchronize brackets the timed region and the
max over ranks is reported.

Prints ONE JSON line (rank 0) with the roofline of the dominant kernel (HIP
events on its stream) and the CPU baseline (oracle restatement of
SIMD-diagonal-maximum on this host's cores, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# gfx950 peaks (MI355X_MICROARCH.md, chip-level parameters / matrix cores)
PEAK_F32_MFMA_TFLOPS = 157.3          # v_mfma_f32_16x16x4_f32, dense
PEAK_I8_MFMA_TOPS = 2 * 2516.6        # i8 MFMA = 2x bf16 dense (2.5 PF)
PEAK_HBM_GBS = 8000.0

MODES = {
    "fp32": ("diagonal-maximum", "f32"),
    "simd": ("SIMD-diagonal-maximum", "s8xs8->i32"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--mode", choices=sorted(MODES), default="fp32")
    p.add_argument("--frames", type=int, default=0, help="frames per GPU per step (default: mode-specific)")
    p.add_argument("--mixtures", type=int, default=5000)
    p.add_argument("--densities", type=int, default=160)
    p.add_argument("--dim", type=int, default=39)
    p.add_argument("--no-best", action="store_true", help="do not write best-density indices")
    p.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--cpu-frames-per-thread", type=int, default=96)
    p.add_argument("--extra-mode", action="store_true", help="also time the other mode (reported under 'modes')")
    return p.parse_args()


def dist_setup(args):
    import torch
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return ws, rank, local


def barrier(ws):
    import torch
    if ws > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x: float, ws: int) -> float:
    if ws == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def load_pmc(mode: str):
    """HBM bytes per launch of the dominant kernel from a committed rocprofv3 PMC summary, or None."""
    path = os.path.join(ROOT, "profiles", f"pmc_{mode}.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    except Exception:
        return None


def run_mode(args, mode, ms, ws, rank, local, frames_per_gpu):
    import torch
    import rasr_amd as ra
    kind, dtype = MODES[mode]
    dev = torch.device("cuda", local)
    sc = ra.Scorer(ms, kind, max_frames=frames_per_gpu, device=local)
    M = sc.n_mixtures()
    frames = torch.from_numpy(ra.synthetic_frames(frames_per_gpu, args.dim, seed=1000 + rank)).to(dev)
    scores = torch.empty((M, frames_per_gpu), dtype=torch.float32, device=dev)
    best = None if args.no_best else torch.empty((M, frames_per_gpu), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    for _ in range(args.warmup):
        sc.score_device(frames, scores, best, stream)
    barrier(ws)
    sc.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sc.score_device(frames, scores, best, stream)
    barrier(ws)
    dt = time.perf_counter() - t0
    kms, nl = sc.kernel_time(reset=True)
    sc.set_timing(False)
    dt_max = max_over_ranks(dt, ws)
    kms_avg = max_over_ranks(kms / max(nl, 1), ws)
    total_frames = ws * frames_per_gpu * args.steps
    n_dens = int(ms.n_entries)
    algo = 2.0 * args.dim * n_dens * frames_per_gpu  # one multiply-add per (frame, density, component)
    peak = PEAK_F32_MFMA_TFLOPS if mode == "fp32" else PEAK_I8_MFMA_TOPS
    achieved = algo / (kms_avg * 1e-3) / 1e12
    out_bytes = M * frames_per_gpu * (4 + (0 if best is None else 4))
    res = {
        "value": total_frames / dt_max,
        "ms_per_step": dt_max / args.steps * 1e3,
        "dtype": dtype,
        "kernel_ms": kms_avg,
        "roofline": {
            "bound": "mfma",
            "achieved": achieved,
            "peak": peak,
            "unit": "TFLOP/s",
            "frac": achieved / peak,
            "traffic": load_pmc(mode),
            "kernel": "scoreI8" if mode == "simd" else "scoreF32",
            "algorithmic_flop_per_launch": algo,
            "output_bytes_per_launch": out_bytes,
        },
    }
    del sc
    return res


def cpu_baseline(args, ms):
    import oracle
    threads = args.cpu_threads or min(16, os.cpu_count() or 1)
    n = threads * args.cpu_frames_per_thread
    import rasr_amd as ra
    frames = ra.synthetic_frames(n, args.dim, seed=999)
    o = oracle.OracleSimd(ms)
    t0 = time.perf_counter()
    o.score(frames, n_threads=threads)
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{n} frames x {ms.n_entries} densities, SIMD-diagonal-maximum restatement "
                      f"(oracle/gmm_oracle.c, SSE2 u8 SSD), {threads} threads, {dt:.1f} s"}


def main():
    args = parse()
    import torch
    import rasr_amd as ra
    ws, rank, local = dist_setup(args)
    frames_per_gpu = args.frames or (8192 if args.mode == "fp32" else 32768)
    ms = ra.synthetic_mixture_set(args.mixtures, args.densities, args.dim, seed=2024)
    res = run_mode(args, args.mode, ms, ws, rank, local, frames_per_gpu)
    extra = {}
    if args.extra_mode:
        other = "simd" if args.mode == "fp32" else "fp32"
        fo = 32768 if other == "simd" else 8192
        r2 = run_mode(args, other, ms, ws, rank, local, fo)
        extra[other] = {"value": r2["value"], "frames_per_gpu": fo, "dtype": r2["dtype"],
                        "scorer": MODES[other][0], "roofline": r2["roofline"]}
    cpu = None
    if rank == 0 and ws == 1 and args.cpu_baseline == "auto":
        cpu = cpu_baseline(args, ms)
    if rank == 0:
        line = {
            "metric": "frames/sec scored, 39-dim x 800k-density diag-GMM",
            "value": res["value"],
            "unit": "frames/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": res["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": res["dtype"],
            "data": "synthetic (SURVEY 8(d): means N(0,1), var 0.5+|N(0,1)|, frames N(0,1))",
            "config": {
                "workload": f"{'800k' if args.mixtures * args.densities == 800000 else args.mixtures * args.densities}"
                            f"-density diag-GMM, {args.dim}-dim, {MODES[args.mode][0]}, batched frames",
                "scorer": MODES[args.mode][0],
                "mixtures": args.mixtures,
                "densities_per_mixture": args.densities,
                "dimension": args.dim,
                "frames_per_gpu_per_step": frames_per_gpu,
                "best_density": not args.no_best,
                "parallelism": f"frame-sharded replicas x{ws}",
            },
            "roofline": res["roofline"],
            "cpu_baseline": cpu,
        }
        if extra:
            line["modes"] = extra
        print(json.dumps(line), flush=True)
    if ws > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
