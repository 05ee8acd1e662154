#!/usr/bin/env python3
"""bench.py -- frames/s of the MI355X diagonal-GMM scorer (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 800k-density triphone diag-GMM, 39-dim,
5000 mixtures x 160 densities, pooled covariance, synthetic model and frames
(SURVEY.md 8(d)); one step = scoring one batch of frames against every mixture
(scores + best densities written to HBM), inputs resident in HBM.  Headline mode
"fp32" is the diagonal-maximum scorer on f32 MFMA (configs[1] says fp32); the
bit-exact SIMD-diagonal-maximum scorer (int8 MFMA) is timed too and reported
under "modes".

  python bench.py [--gpus N] [--steps K] [--warmup W] [--mode fp32|simd] [--frames F]
                  [--parallel frames|mixtures|densities]

N > 1 is launched by torch.distributed.run, one process per GPU:
  --parallel frames   (default; configs 2-3): every rank scores its own F frames
                      against a replica of the model, no collective on the data
                      path, "scaling": "weak";
  --parallel mixtures (config 4): every rank holds 1/N of the mixtures (density
                      balanced) and scores the same F frames; the [M][F] score
                      table is assembled with one all-gather over RCCL per step,
                      "scaling": "strong";
  --parallel densities (config 4 as written): every rank holds 1/N of the densities
                      (mixtures on shard boundaries split between ranks) and scores
                      the same F frames; whole mixtures all-gathered, split ones
                      reduced per frame with an RCCL all-reduce(MIN), "strong".
A barrier + synchronize brackets the timed region; the max over ranks is reported.

Prints ONE JSON line (rank 0) with the roofline of the dominant kernel (HIP events
on its stream) and the CPU baseline (oracle restatement of SIMD-diagonal-maximum
on this host's cores, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# gfx950 peaks (MI355X_MICROARCH.md, chip-level parameters / matrix cores)
PEAK_F32_MFMA_TFLOPS = 157.3          # v_mfma_f32_16x16x4_f32, dense
PEAK_F16_MFMA_TFLOPS = 2516.6         # v_mfma_f32_16x16x32_f16, dense (same rate as bf16)
PEAK_I8_MFMA_TOPS = 2 * 2516.6        # i8 MFMA = 2x the bf16 dense rate
SPLIT_PRODUCTS = 3                    # split-f16 kernel: mh*xh + mh*xl + ml*xh per f32 multiply-add

MODES = {
    "fp32": ("diagonal-maximum", "f32"),
    "simd": ("SIMD-diagonal-maximum", "s8xs8->i32 (u8-quantized, bit-exact)"),
    "sum": ("diagonal-sum", "f32"),  # log-sum-exp variant (GaussDiagonalSumFeatureScorer), --mode sum
    "nn": ("nn-batch-feature-scorer", "bf16 x bf16 -> f32 (MFMA), f32 bias/activation"),  # config 5, --mode nn
    # density preselection (256 clusters, 32 selected per frame): cluster selection + masked scoring
    "presel-float": ("preselection-batch-float", "f32"),
    "presel-int": ("preselection-batch-int", "s8xs8->i32 (u8-quantized, bit-exact)"),
}
DEFAULT_FRAMES = {"fp32": 32768, "simd": 32768, "sum": 32768, "nn": 32768, "presel-float": 32768,
                  "presel-int": 32768}  # frames per GPU per step (batch)
# BASELINE config 5 network (hybrid DNN): 11 x 39 spliced MFCC input, 6 sigmoid layers of 2048, 5000 classes
NN_DIMS = [429] + [2048] * 6 + [5000]


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--mode", choices=sorted(MODES), default="fp32")
    p.add_argument("--frames", type=int, default=0, help="frames per GPU per step (default: mode-specific)")
    p.add_argument("--parallel", choices=["frames", "mixtures", "densities"], default="frames")
    p.add_argument("--mixtures", type=int, default=5000)
    p.add_argument("--densities", type=int, default=160)
    p.add_argument("--dim", type=int, default=39)
    p.add_argument("--no-best", action="store_true", help="do not write best-density indices")
    p.add_argument("--no-extra-mode", action="store_true", help="do not time the other mode")
    p.add_argument("--native-f32", action="store_true",
                   help="fp32 mode on the f32-MFMA kernel instead of the split-f16 kernel")
    p.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--cpu-frames-per-thread", type=int, default=3000)
    return p.parse_args()


def dist_setup():
    """One process per GPU over RCCL ("nccl").  Rehearsal only (not used by the driver): with
    RASR_BENCH_SAME_DEVICE=1 every rank uses GPU 0 and RASR_BENCH_BACKEND=gloo replaces RCCL, so the
    N > 1 flow can be exercised on a one-GPU box."""
    import torch
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("RASR_BENCH_SAME_DEVICE") == "1":
        local = 0
    if ws > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        backend = os.environ.get("RASR_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
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
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summary
    (scripts/pmc_summary.py: FETCH_SIZE doubled per the gfx950 correction + WRITE_SIZE)."""
    path = os.path.join(ROOT, "profiles", f"pmc_{mode}.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def run_mode(args, mode, ms, ws, rank, local, frames_per_gpu):
    import torch
    import rasr_amd as ra
    from rasr_amd import parallel
    kind, dtype = MODES[mode]
    dev = torch.device("cuda", local)
    sharded = args.parallel in ("mixtures", "densities") and ws > 1
    if sharded:
        if args.parallel == "densities":
            scorer = parallel.DensityShardedScorer(ms, kind, frames_per_gpu, rank, ws, device=local)
        else:
            scorer = parallel.MixtureShardedScorer(ms, kind, frames_per_gpu, rank, ws, device=local)
        sc = scorer.scorer
        seed = 1000  # every rank scores the same frames
    else:
        sc = ra.Scorer(ms, kind, max_frames=frames_per_gpu, device=local,
                       native_f32=args.native_f32 and mode == "fp32")
        seed = 1000 + rank
    m_local = sc.n_mixtures()
    frames = torch.from_numpy(ra.synthetic_frames(frames_per_gpu, args.dim, seed=seed)).to(dev)
    scores = torch.empty((m_local, frames_per_gpu), dtype=torch.float32, device=dev)
    best = None if (args.no_best or mode.startswith("presel")) else torch.empty((m_local, frames_per_gpu), dtype=torch.int32,
                                                                                   device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        if sharded:
            scorer.score(frames, scores, best, stream)  # score own mixtures + all-gather the table
        else:
            sc.score_device(frames, scores, best, stream)

    for _ in range(args.warmup):
        step()
    barrier(ws)
    sc.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier(ws)
    dt = time.perf_counter() - t0
    kms, nl = sc.kernel_time(reset=True)
    sc.set_timing(False)
    dt_max = max_over_ranks(dt, ws)
    kms_avg = max_over_ranks(kms / max(nl, 1), ws)
    total_frames = (1 if sharded else ws) * frames_per_gpu * args.steps
    if sharded and args.parallel == "densities":
        d_local = scorer.shards[rank]["entries"][1] - scorer.shards[rank]["entries"][0]
    elif sharded:
        d_local = int(ms.mixture_offsets[min(ms.n_mixtures, scorer.shards[rank][1])]
                      - ms.mixture_offsets[scorer.shards[rank][0]])
    else:
        d_local = int(ms.n_entries)
    algo = 2.0 * args.dim * d_local * frames_per_gpu  # one multiply-add per (frame, density, component)
    kernel = sc.main_kernel()
    split = kernel in ("scoreSplit", "scoreSplit32", "scoreSplitSum")
    if split:
        # f32-accurate contraction on the f16 matrix cores: 3 f16 products per f32 multiply-add, so the
        # roofline for this arithmetic is the dense f16 peak / 3; the MFMA work actually issued covers
        # K = 3 D + 7 (row-constant and ||x'||^2 limbs) padded to the K step (32 for 16x16x32, 16 for
        # 32x32x16) per (frame, density)
        peak = PEAK_F16_MFMA_TFLOPS / SPLIT_PRODUCTS
        kq = 16 if kernel == "scoreSplit32" else 32
        k_issued = kq * ((3 * args.dim + 7 + kq - 1) // kq)
        issued = 2.0 * k_issued * d_local * frames_per_gpu
    elif mode in ("fp32", "sum"):
        peak = PEAK_F32_MFMA_TFLOPS
        issued = 2.0 * 4 * ((args.dim + 1 + 3) // 4) * d_local * frames_per_gpu
    else:
        peak = PEAK_I8_MFMA_TOPS
        issued = 2.0 * 64 * ((args.dim + 63) // 64) * d_local * frames_per_gpu
    sec = kms_avg * 1e-3
    achieved = algo / sec / 1e12
    res = {
        "value": total_frames / dt_max,
        "ms_per_step": dt_max / args.steps * 1e3,
        "dtype": dtype if not split else
        "f32 (operands split into 2 f16 pieces, 3 f16 MFMA products, f32 accumulate)",
        "frames_per_gpu": frames_per_gpu,
        "roofline": {
            "bound": "mfma",
            "achieved": achieved,
            "peak": peak,
            "unit": "TFLOP/s",
            "frac": achieved / peak,
            "traffic": load_pmc(mode) if not sharded else None,
            "kernel": kernel,
            "kernel_ms": kms_avg,
            "algorithmic_flop_per_launch": algo,
            "issued_mfma_flop_per_launch": issued,
            "issued_mfma_tflops": issued / sec / 1e12,
            "issued_mfma_frac_of_dtype_peak": issued / sec / 1e12 / (
                PEAK_F16_MFMA_TFLOPS if split else peak),
            "output_bytes_per_launch": m_local * frames_per_gpu * (4 + (0 if best is None else 4)),
        },
    }
    del sc
    return res


def run_nn(args, ws, rank, local, frames_per_gpu):
    """Nn::BatchFeatureScorer drop-in (rasr_amd.nn): one bf16 MFMA GEMM per layer, bias + activation fused;
    a step scores frames_per_gpu frames on every rank (frame-sharded replicas, no collective)."""
    import numpy as np
    import torch
    import rasr_amd as ra
    from rasr_amd import nn
    dev = torch.device("cuda", local)
    layers = nn.synthetic_network(NN_DIMS, "sigmoid", seed=2024)
    lp = np.full(NN_DIMS[-1], -np.log(NN_DIMS[-1]), np.float32)
    sc = nn.NnScorer(layers, log_prior=lp, prior_scale=1.0, max_frames=frames_per_gpu, device=local)
    frames = torch.from_numpy(ra.synthetic_frames(frames_per_gpu, NN_DIMS[0], seed=1000 + rank)).to(dev)
    scores = torch.empty((NN_DIMS[-1], frames_per_gpu), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    for _ in range(args.warmup):
        sc.score_device(frames, scores, stream)
    barrier(ws)
    sc.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sc.score_device(frames, scores, stream)
    barrier(ws)
    dt = time.perf_counter() - t0
    kms, nl = sc.kernel_time(reset=True)
    sc.set_timing(False)
    dt_max = max_over_ranks(dt, ws)
    kms_avg = max_over_ranks(kms / max(nl, 1), ws)
    algo = 2.0 * sum(a * b for a, b in zip(NN_DIMS[:-1], NN_DIMS[1:])) * frames_per_gpu
    pad = lambda x, q: (x + q - 1) // q * q  # GEMM tiles: outputs to 128, the input to 64
    kp = [pad(NN_DIMS[0], 64)] + [pad(d, 128) for d in NN_DIMS[1:-1]]
    issued = 2.0 * sum(k * pad(m, 128) for k, m in zip(kp, NN_DIMS[1:])) * pad(frames_per_gpu, 128)
    sec = kms_avg * 1e-3
    return {
        "value": ws * frames_per_gpu * args.steps / dt_max,
        "ms_per_step": dt_max / args.steps * 1e3,
        "dtype": MODES["nn"][1],
        "frames_per_gpu": frames_per_gpu,
        "roofline": {
            "bound": "mfma", "achieved": algo / sec / 1e12, "peak": PEAK_F16_MFMA_TFLOPS, "unit": "TFLOP/s",
            "frac": algo / sec / 1e12 / PEAK_F16_MFMA_TFLOPS, "traffic": None, "kernel": "nnGemm8p",
            "kernel_ms": kms_avg, "algorithmic_flop_per_launch": algo, "issued_mfma_flop_per_launch": issued,
            "issued_mfma_tflops": issued / sec / 1e12,
        },
    }


def cpu_baseline(args, ms):
    import oracle
    import rasr_amd as ra
    threads = args.cpu_threads or min(16, os.cpu_count() or 1)
    n = threads * args.cpu_frames_per_thread
    frames = ra.synthetic_frames(n, args.dim, seed=999)
    o = oracle.OracleSimd(ms)
    t0 = time.perf_counter()
    o.score(frames, n_threads=threads)
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{n} frames x {ms.n_entries} densities, SIMD-diagonal-maximum restatement "
                      f"(oracle/gmm_oracle.c, SSE2 u8 SSD like the reference JIT), {threads} threads, {dt:.1f} s"}


def main():
    args = parse()
    import rasr_amd as ra
    ws, rank, local = dist_setup()
    frames_per_gpu = args.frames or DEFAULT_FRAMES[args.mode]
    if args.mode == "nn":
        res = run_nn(args, ws, rank, local, frames_per_gpu)
        if rank == 0:
            print(json.dumps({
                "metric": "frames/sec scored, hybrid-DNN posteriors (Nn::BatchFeatureScorer)", "value": res["value"],
                "unit": "frames/s", "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": res["ms_per_step"], "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                "dtype": res["dtype"], "data": "synthetic (random-init network, frames N(0,1))",
                "config": {"workload": "hybrid DNN " + "-".join(map(str, NN_DIMS)) + " sigmoid, 5000 classes",
                           "frames_per_gpu_per_step": frames_per_gpu,
                           "parallelism": f"frame-sharded replicas x{ws}"},
                "roofline": res["roofline"], "cpu_baseline": None}), flush=True)
        if ws > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    ms = ra.synthetic_mixture_set(args.mixtures, args.densities, args.dim, seed=2024)
    res = run_mode(args, args.mode, ms, ws, rank, local, frames_per_gpu)
    extra = {}
    if not args.no_extra_mode:
        other = "simd" if args.mode != "simd" else "fp32"  # (nn returned above)
        r2 = run_mode(args, other, ms, ws, rank, local, DEFAULT_FRAMES[other])
        extra[other] = {"value": r2["value"], "ms_per_step": r2["ms_per_step"],
                        "frames_per_gpu_per_step": r2["frames_per_gpu"], "dtype": r2["dtype"],
                        "scorer": MODES[other][0], "roofline": r2["roofline"]}
    cpu = None
    if rank == 0 and ws == 1 and args.cpu_baseline == "auto":
        cpu = cpu_baseline(args, ms)
    if rank == 0:
        n_dens = args.mixtures * args.densities
        line = {
            "metric": "frames/sec scored, 39-dim x 800k-density diag-GMM",
            "value": res["value"],
            "unit": "frames/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": res["ms_per_step"],
            "higher_is_better": True,
            "scaling": "strong" if (args.parallel in ("mixtures", "densities") and ws > 1) else "weak",
            "vs_baseline": None,
            "dtype": res["dtype"],
            "data": "synthetic (SURVEY 8(d): means N(0,1), var 0.5+|N(0,1)|, frames N(0,1))",
            "config": {
                "workload": f"{n_dens // 1000}k-density diag-GMM, {args.dim}-dim, {MODES[args.mode][0]}, "
                            f"batched frames",
                "scorer": MODES[args.mode][0],
                "mixtures": args.mixtures,
                "densities_per_mixture": args.densities,
                "dimension": args.dim,
                "frames_per_gpu_per_step": frames_per_gpu,
                "best_density": not args.no_best and not args.mode.startswith("presel"),
                "parallelism": (f"mixture-sharded x{ws} + RCCL all-gather" if args.parallel == "mixtures" and ws > 1
                                else f"density-sharded x{ws} + RCCL all-reduce(MIN) of split mixtures + all-gather"
                                if args.parallel == "densities" and ws > 1 else f"frame-sharded replicas x{ws}"),
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
