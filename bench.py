#!/usr/bin/env python3
"""bench.py -- frames/s of the MI355X diagonal-GMM scorer (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 800k-density triphone diag-GMM, 39-dim,
5000 mixtures x 160 densities, pooled covariance, synthetic model and frames
(SURVEY.md 8(d)); inputs resident in HBM.  One step scores a block of frames
against every mixture (scores + best densities written to HBM): `--launches`
scorer calls of `--frames` frames each (32768 by default), on consecutive frame
slices into consecutive columns of one [mixtures][frames per step] table, so 20
steps time >= 1 s of steady state (the loop is power-bound; a 0.1 s window reads
the boost clock).  Headline mode "fp32" is the diagonal-maximum scorer
(configs[1] says fp32); the bit-exact SIMD-diagonal-maximum scorer (int8 MFMA)
is timed too and reported under "modes".

  python bench.py [--gpus N] [--steps K] [--warmup W] [--mode fp32|simd|...] [--frames F]
                  [--launches L] [--parallel frames|mixtures|densities]

--gpus N > 1 without WORLD_SIZE in the environment: this process starts
`torch.distributed.run --nproc-per-node N bench.py ...` as a child (before any
GPU call), relays its output and exits with its code; every rank checks that
the world it joined has N ranks.  Layouts (one process per GPU, RCCL):
  --parallel frames   (default; configs 2-3): every rank scores its own frames
                      against a replica of the model, no collective on the data
                      path, "scaling": "weak";
  --parallel mixtures: every rank holds 1/N of the mixtures (density balanced) and
                      scores the same frames; the table is assembled with one
                      all-gather per launch, "scaling": "strong";
  --parallel densities (config 4 as written): every rank holds 1/N of the densities
                      (mixtures on shard boundaries split between ranks) and scores
                      the same frames; whole mixtures all-gathered, split ones
                      reduced per frame with an RCCL all-reduce(MIN), "strong".
A barrier + synchronize brackets the timed region; the max over ranks is reported.

Prints ONE JSON line (rank 0) with the roofline of the dominant kernel (HIP events
on its stream, averaged over every launch of the timed region), the CPU baseline
(oracle restatements of SIMD-diagonal-maximum and diagonal-maximum on this host,
rank 0 at N=1 only) and the host-buffer boundary rate (gmm_score_host into a
page-locked table, PCIe included; never `value`).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import signal
import socket
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# gfx950 peaks (MI355X_MICROARCH.md, chip-level parameters / matrix cores)
PEAK_F32_MFMA_TFLOPS = 157.3          # v_mfma_f32_16x16x4_f32, dense
PEAK_F16_MFMA_TFLOPS = 2516.6         # v_mfma_f32_16x16x32_f16, dense (same rate as bf16)
PEAK_I8_MFMA_TOPS = 2 * 2516.6        # i8 MFMA = 2x the bf16 dense rate
SPLIT_PRODUCTS = 3                    # split-f16 kernel: mh*xh + mh*xl + ml*xh per f32 multiply-add
CPU_SHARE_PER_GPU = 16                # host CPUs a one-GPU box grants this job
N_SIMDS = 256 * 4                     # 256 CUs x 4 SIMDs
CLOCK_GHZ = 2.4                       # peak engine clock the MFMA peaks are quoted at
VOP3_CYCLES = 3.14                    # measured issue cost of a 3-source VOP3 per SIMD (profiles/r02/vgpr_banks.txt)

MODES = {
    "fp32": ("diagonal-maximum", "f32"),
    "simd": ("SIMD-diagonal-maximum", "s8xs8->i32 (u8-quantized, bit-exact)"),
    # batched int scorer (no best densities): the score-only class layout (gmm_prepare.cc buildClassLayout)
    "bint": ("batch-diagonal-maximum-int", "s8xs8->i32 (u8-quantized, bit-exact)"),
    # the assigning scorers without best densities (the search reads only score(e)): SIMD on its score-only
    # twin (class layout), fp32 without the index tag
    "simd-scores": ("SIMD-diagonal-maximum", "s8xs8->i32 (u8-quantized, bit-exact)"),
    "fp32-scores": ("diagonal-maximum", "f32"),
    "sum": ("diagonal-sum", "f32"),  # log-sum-exp variant (GaussDiagonalSumFeatureScorer), --mode sum
    "nn": ("nn-batch-feature-scorer", "bf16 x bf16 -> f32 (MFMA), f32 bias/activation"),  # config 5, --mode nn
    # density preselection (256 clusters, 32 selected per frame): cluster selection + masked scoring
    "presel-float": ("preselection-batch-float", "f32"),
    "presel-int": ("preselection-batch-int", "s8xs8->i32 (u8-quantized, bit-exact)"),
}
FRAMES_PER_LAUNCH = 32768  # frames per scorer call (the scorer's max_frames)
# scorer calls per step: about 50-60 ms of GPU work per step at the measured rates, so 20 steps >= 1 s
DEFAULT_LAUNCHES = {"fp32": 12, "simd": 32, "bint": 40, "simd-scores": 40, "fp32-scores": 12, "sum": 8, "nn": 16, "presel-float": 8, "presel-int": 8}
# BASELINE config 5 network (hybrid DNN): 11 x 39 spliced MFCC input, 6 sigmoid layers of 2048, 5000 classes
NN_DIMS = [429] + [2048] * 6 + [5000]
# N > 1 budget (the driver kills a run at 600 s): the headline and the other modes first (~1-2 min at N = 8), then
# the checks of never-executed multi-GPU paths, each in child processes killed at FENCE_TIMEOUT_S; whatever still
# runs at DEADLINE_S, the JSON line is printed with the extras that finished and every rank exits 0.
FENCE_TIMEOUT_S = float(os.environ.get("RASR_BENCH_FENCE_TIMEOUT_S", 150))
DEADLINE_S = 480.0
PG_TIMEOUT_S = 180  # the ranks' process group: a collective that hangs aborts the rank instead of outliving the run


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--mode", choices=sorted(MODES), default="fp32")
    p.add_argument("--frames", type=int, default=0, help=f"frames per scorer call (default {FRAMES_PER_LAUNCH})")
    p.add_argument("--launches", type=int, default=0, help="scorer calls per step (default: mode-specific)")
    p.add_argument("--parallel", choices=["frames", "mixtures", "densities"], default="frames")
    p.add_argument("--mixtures", type=int, default=5000)
    p.add_argument("--densities", type=int, default=160)
    p.add_argument("--dim", type=int, default=39)
    p.add_argument("--ragged", action="store_true",
                   help="SURVEY 8(d) ragged variant: K_m ~ U[64, 256] with the same total of densities")
    p.add_argument("--tying", choices=["pooled", "mixture-specific", "none"], default="pooled",
                   help="covariance tying of the synthetic model (RASR covariance-tying; the configs are pooled)")
    p.add_argument("--no-best", action="store_true", help="do not write best-density indices")
    p.add_argument("--no-extra-mode", action="store_true", help="do not time the other mode")
    p.add_argument("--nn-activation", default="sigmoid", choices=["sigmoid", "tanh", "relu", "elu", "identity"],
                   help="--mode nn: hidden-layer activation (config 5 is sigmoid)")
    p.add_argument("--no-density-check", action="store_true",
                   help="N > 1: skip the density-sharded (config 4, RCCL) check beside the headline")
    p.add_argument("--native-f32", action="store_true",
                   help="fp32 mode on the f32-MFMA kernel instead of the split-f16 kernel")
    p.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    p.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (default: the CPUs available)")
    p.add_argument("--cpu-frames-per-thread", type=int, default=3000)
    p.add_argument("--host-boundary", choices=["auto", "off"], default="auto")
    p.add_argument("--capi-sharded-child", default="",
                   help="internal: run the C-ABI density-sharded check over these comma-separated devices in this "
                        "process (started by rank 0 of an N > 1 run) and print one JSON record")
    p.add_argument("--density-check-child", action="store_true",
                   help="internal: one rank of the fenced density-sharded (config 4, RCCL) check, started by rank 0 "
                        "of an N > 1 run; rank 0 of the check prints one JSON record")
    p.add_argument("--extras", choices=["auto", "off"], default="auto",
                   help="N = 1: device lines at 256/1024/4096 frames per call and the C++ drop-in protocol record")
    p.add_argument("--deadline", type=float, default=float(os.environ.get("RASR_BENCH_DEADLINE_S", DEADLINE_S)),
                   help="seconds after start at which the JSON line is printed with whatever extras have finished "
                        "and every rank exits (0: no deadline)")
    return p.parse_args()


# ---------------------------------------------------------------------------
# launcher: --gpus N without a torch.distributed environment
# ---------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """Run this script as N ranks under torch.distributed.run (a child process; nothing here has touched the
    GPU) and return its exit code.  The child's stdout (rank 0's JSON line) passes through unchanged."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this pool
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


def fence_probe() -> bool:
    """RASR_BENCH_FENCE_PROBE=1 (tests/test_bench_fence.py, CPU): the N > 1 orchestration -- process group, fenced
    children, deadline, the line -- with a synthetic headline and synthetic check payloads, no GPU work;
    RASR_BENCH_INJECT=hang@R | raise@R | capi-hang | parent-hang@R injects a fault on rank R."""
    return os.environ.get("RASR_BENCH_FENCE_PROBE") == "1"


def _inject(what: str, rank: int) -> None:
    """Probe mode only: RASR_BENCH_INJECT=<what>@<rank> (or <what> for every rank) raises ("raise") or hangs."""
    spec = os.environ.get("RASR_BENCH_INJECT", "")
    if not fence_probe() or not spec:
        return
    kind, _, r = spec.partition("@")
    if kind == what and (r == "" or int(r) == rank):
        if what == "raise":
            raise RuntimeError(f"injected fault ({spec}) on rank {rank}")
        while True:  # an injected hang: as a rank stuck in a collective whose peer never arrives
            time.sleep(1)


def dist_setup(args):
    """One process per GPU over RCCL ("nccl"), the process group with an explicit timeout (PG_TIMEOUT_S).
    Rehearsal only (not used by the driver): with RASR_BENCH_SAME_DEVICE=1 every rank uses GPU 0 and
    RASR_BENCH_BACKEND=gloo replaces RCCL, so the N > 1 flow can be exercised on a one-GPU box."""
    import datetime
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}")
    if os.environ.get("RASR_BENCH_SAME_DEVICE") == "1":
        local = 0
    timeout = datetime.timedelta(seconds=PG_TIMEOUT_S)
    if fence_probe():
        if ws > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo", timeout=timeout)
        return ws, rank, local
    import torch
    if ws > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        backend = os.environ.get("RASR_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timeout)
        else:
            dist.init_process_group(backend, timeout=timeout)
        seen = dist.get_world_size()
        if seen != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the process group has {seen} ranks")
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


def _kernel_id() -> str:
    from rasr_amd import _capi
    return _capi.load_library().gmm_kernel_id().decode()


def load_pmc(mode: str, frames_per_launch: int, default_model: bool = True):
    """HBM bytes per launch of the dominant kernel from the rocprofv3 PMC summary under profiles/
    (scripts/pmc_summary.py: FETCH_SIZE doubled per the gfx950 correction + WRITE_SIZE), used only when it
    was collected on this build's kernels (gmm_kernel_id) at this launch size and on the model the summaries are
    profiled on (scripts/profile_pmc.sh: the default 39-dim, 160-density bench model); else null."""
    path = os.path.join(ROOT, "profiles", f"pmc_{mode}.json")
    if not default_model:
        return None, f"{os.path.relpath(path, ROOT)} is profiled on the default model, not this one"
    try:
        with open(path) as f:
            pmc = json.load(f)
    except (OSError, ValueError):
        return None, None
    if pmc.get("kernel_id") != _kernel_id() or pmc.get("frames_per_launch") != frames_per_launch:
        return None, f"{os.path.relpath(path, ROOT)} is from other kernels or another launch size"
    return pmc.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)


def _step_slices(total: int, per: int):
    return [(i, min(i + per, total)) for i in range(0, total, per)]


def run_mode(args, mode, ms, ws, rank, local, launches):
    import torch
    import rasr_amd as ra
    from rasr_amd import parallel
    kind, dtype = MODES[mode]
    dev = torch.device("cuda", local)
    fpl = args.frames or FRAMES_PER_LAUNCH
    f_step = fpl * launches
    sharded = args.parallel in ("mixtures", "densities") and ws > 1
    if sharded:
        if args.parallel == "densities":
            scorer = parallel.DensityShardedScorer(ms, kind, fpl, rank, ws, device=local)
        else:
            scorer = parallel.MixtureShardedScorer(ms, kind, fpl, rank, ws, device=local)
        sc = scorer.scorer
        seed = 1000  # every rank scores the same frames
    else:
        sc = ra.Scorer(ms, kind, max_frames=fpl, device=local, native_f32=args.native_f32 and mode == "fp32")
        seed = 1000 + rank
    m_local = sc.n_mixtures()
    frames = torch.from_numpy(ra.synthetic_frames(f_step, args.dim, seed=seed)).to(dev)
    # batch types: no best; the -scores modes: the assigning types asked for scores only
    want_best = not (args.no_best or mode.startswith("presel") or mode == "bint" or mode.endswith("-scores"))
    scores = torch.empty((m_local, f_step if not sharded else fpl), dtype=torch.float32, device=dev)
    best = (torch.empty((m_local, f_step if not sharded else fpl), dtype=torch.int32, device=dev)
            if want_best else None)
    stream = torch.cuda.current_stream(dev)
    slices = _step_slices(f_step, fpl)

    def step():
        for a, b in slices:
            if sharded:  # this rank's mixtures / densities + the collectives, per launch
                scorer.score(frames[a:b], scores, best, stream)
            else:
                sc.score_device(frames[a:b], scores[:, a:b], None if best is None else best[:, a:b], stream)

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
    total_frames = (1 if sharded else ws) * f_step * args.steps
    if sharded and args.parallel == "densities":
        d_local = scorer.shards[rank]["entries"][1] - scorer.shards[rank]["entries"][0]
    elif sharded:
        d_local = int(ms.mixture_offsets[min(ms.n_mixtures, scorer.shards[rank][1])]
                      - ms.mixture_offsets[scorer.shards[rank][0]])
    else:
        d_local = int(ms.n_entries)
    algo = 2.0 * args.dim * d_local * fpl  # one multiply-add per (frame, density, component), per launch
    kernel = sc.main_kernel()
    split = kernel in ("scoreSplit", "scoreSplitWide", "scoreSplit32", "scoreSplitSum", "scoreSplit32Sum")
    if split:
        # f32-accurate contraction on the f16 matrix cores: 3 f16 products per f32 multiply-add, so the
        # roofline for this arithmetic is the dense f16 peak / 3; the MFMA work actually issued covers
        # K = 3 D + 7 (row-constant and ||x'||^2 limbs) padded to the K step (32 for 16x16x32, 16 for
        # 32x32x16) per (frame, density)
        peak = PEAK_F16_MFMA_TFLOPS / SPLIT_PRODUCTS
        kq = 16 if kernel in ("scoreSplit32", "scoreSplit32Sum") else 32
        k_issued = kq * ((3 * args.dim + 7 + kq - 1) // kq)
        issued = 2.0 * k_issued * d_local * fpl
    elif mode in ("fp32", "fp32-scores", "sum"):
        peak = PEAK_F32_MFMA_TFLOPS
        issued = 2.0 * 4 * ((args.dim + 1 + 3) // 4) * d_local * fpl
    else:
        peak = PEAK_I8_MFMA_TOPS
        issued = 2.0 * 64 * ((args.dim + 63) // 64) * d_local * fpl
    sec = kms_avg * 1e-3
    achieved = algo / sec / 1e12
    default_model = (args.dim == 39 and not args.ragged and args.mixtures == 5000 and args.densities == 160
                     and args.tying == "pooled")
    traffic, traffic_src = load_pmc(mode, fpl, default_model) if not sharded else (None, None)
    res = {
        "value": total_frames / dt_max,
        "ms_per_step": dt_max / args.steps * 1e3,
        "dtype": dtype if not split else
        "f32 (operands split into 2 f16 pieces, 3 f16 MFMA products, f32 accumulate)",
        "frames_per_step": f_step,
        "frames_per_launch": fpl,
        "launches_per_step": launches,
        "timed_region_s": dt_max,
        "roofline": {
            "bound": "mfma",
            "achieved": achieved,
            "peak": peak,
            "unit": "TFLOP/s",
            "frac": achieved / peak,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": kernel,
            "kernel_ms": kms_avg,
            "kernel_launches_timed": nl,
            "algorithmic_flop_per_launch": algo,
            "issued_mfma_flop_per_launch": issued,
            "issued_mfma_tflops": issued / sec / 1e12,
            "issued_mfma_frac_of_dtype_peak": issued / sec / 1e12 / (
                PEAK_F16_MFMA_TFLOPS if split else peak),
            "output_bytes_per_launch": m_local * fpl * (4 + (0 if best is None else 4)),
        },
    }
    if kernel in ("scoreSplitSum", "scoreSplit32Sum"):
        # diagonal-sum's epilogue is VALU issue-bound: per (frame, density) v_fma + v_exp_f32 + v_add_f32 (4 + 8 + 4
        # cycles per wave64 instruction), the key v_and_or_b32 (4) and half a v_min3 (2) with best densities, plus
        # the cycles the MFMAs hold the vector issue (8 per 32x32x16 over 16 K: 4 per 64 values at K = 128; 8 per
        # 16x16x32 over 32 K: 8 per 64 values)
        cyc = (16 + (6 if best is not None else 2)) + (4 if kernel == "scoreSplit32Sum" else 8)
        ceiling = N_SIMDS * CLOCK_GHZ * 1e9 * 64.0 / (cyc * d_local)
        res["roofline"]["valu"] = {
            "ceiling_frames_per_s": ceiling,
            "frac": (fpl / sec) / ceiling,
            "basis": f"{cyc} issue cycles per 64 (frame, density) values per SIMD (MI355X_MICROARCH.md issue costs), "
                     f"{N_SIMDS} SIMDs at {CLOCK_GHZ} GHz",
        }
    if kernel.startswith("scoreI8"):
        # the quantized scorer is reported against max(t_MFMA, t_VALU).  Its epilogue is one
        # 3-source VOP3 (v_lshl_add) per (frame, density) plus half a v_min3; a wave64 VOP3 issues every
        # VOP3_CYCLES cycles per SIMD with 4 waves per SIMD (scripts/debug/vgpr_banks.hip)
        # The score-only class layout (batch types) has no pack: half a v_min3 per (frame, density)
        # Round 6: plus the vector-issue cycles the MFMAs hold (v_mfma_i32_16x16x64_i8 holds 8 of its 16 cycles,
        # MI355X_MICROARCH.md issue costs; one MFMA per K step of 64 yields 4 values per lane), so the ceiling is
        # the SIMD's whole issue budget, not the epilogue's alone
        # The bound is the larger of that issue time and the MFMA pipe's own 4 cycles per 64 values and K step (the
        # score-only kernels, 0.5 VOP3 per value, are MFMA-bound by it)
        vop3 = 0.5 if (mode == "bint" or (mode == "simd-scores" and best is None)) else 1.5
        ksteps = (args.dim + 63) // 64
        hold = 2.0 * ksteps
        issue = vop3 * VOP3_CYCLES + hold
        cycles = max(issue, 4.0 * ksteps)
        keys_per_s = N_SIMDS * CLOCK_GHZ * 1e9 * 64.0 / cycles
        ceiling = keys_per_s / d_local
        res["roofline"]["valu"] = {
            "ceiling_frames_per_s": ceiling,
            "frac": (fpl / sec) / ceiling,
            "basis": f"max(issue, MFMA pipe) per 64 values per SIMD: {vop3} VOP3 per (frame, density) at "
                     f"{VOP3_CYCLES} cycles plus {hold:g} cycles held by the MFMAs = {issue:.2f}, the MFMAs "
                     f"{4.0 * ksteps:g}; {N_SIMDS} SIMDs at {CLOCK_GHZ} GHz",
        }
    del sc, scores, best, frames
    torch.cuda.empty_cache()
    return res


def run_nn(args, ws, rank, local, launches):
    """Nn::BatchFeatureScorer drop-in (rasr_amd.nn): one bf16 MFMA GEMM per layer, bias + activation fused;
    a step scores launches x frames on every rank (frame-sharded replicas, no collective)."""
    import numpy as np
    import torch
    import rasr_amd as ra
    from rasr_amd import nn
    dev = torch.device("cuda", local)
    fpl = args.frames or FRAMES_PER_LAUNCH
    f_step = fpl * launches
    layers = nn.synthetic_network(NN_DIMS, args.nn_activation, seed=2024)
    lp = np.full(NN_DIMS[-1], -np.log(NN_DIMS[-1]), np.float32)
    sc = nn.NnScorer(layers, log_prior=lp, prior_scale=1.0, max_frames=fpl, device=local)
    frames = torch.from_numpy(ra.synthetic_frames(f_step, NN_DIMS[0], seed=1000 + rank)).to(dev)
    scores = torch.empty((NN_DIMS[-1], f_step), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    slices = _step_slices(f_step, fpl)

    def step():
        for a, b in slices:
            sc.score_device(frames[a:b], scores[:, a:b], stream)

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
    algo = 2.0 * sum(a * b for a, b in zip(NN_DIMS[:-1], NN_DIMS[1:])) * fpl
    pad = lambda x, q: (x + q - 1) // q * q  # GEMM tiles: outputs to 256, the input to 64
    kp = [pad(NN_DIMS[0], 64)] + [pad(d, 256) for d in NN_DIMS[1:-1]]
    issued = 2.0 * sum(k * pad(m, 256) for k, m in zip(kp, NN_DIMS[1:])) * pad(fpl, 256)
    sec = kms_avg * 1e-3
    return {
        "value": ws * f_step * args.steps / dt_max,
        "ms_per_step": dt_max / args.steps * 1e3,
        "dtype": MODES["nn"][1],
        "frames_per_step": f_step,
        "frames_per_launch": fpl,
        "launches_per_step": launches,
        "timed_region_s": dt_max,
        "roofline": {
            "bound": "mfma", "achieved": algo / sec / 1e12, "peak": PEAK_F16_MFMA_TFLOPS, "unit": "TFLOP/s",
            "frac": algo / sec / 1e12 / PEAK_F16_MFMA_TFLOPS, "traffic": None, "kernel": "nnGemm8p (all layers)",
            "kernel_ms": kms_avg, "algorithmic_flop_per_launch": algo, "issued_mfma_flop_per_launch": issued,
            "issued_mfma_tflops": issued / sec / 1e12,
        },
    }


# ---------------------------------------------------------------------------
# CPU baseline and host boundary (rank 0, N = 1)
# ---------------------------------------------------------------------------
def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def available_cpus():
    """(threads to use, note): the CPUs this process may run on -- affinity, capped by a cgroup CPU quota and by
    the per-GPU CPU share of the GPU box (CPU_SHARE_PER_GPU; os.cpu_count() reports the whole machine there)."""
    n = len(os.sched_getaffinity(0))
    note = f"{n} CPUs in the affinity mask"
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            quota = max(1, math.ceil(int(q) / int(p)))
            if quota < n:
                n, note = quota, f"cgroup quota {quota} CPUs"
    except (OSError, ValueError):
        pass
    if n > CPU_SHARE_PER_GPU:
        n, note = CPU_SHARE_PER_GPU, f"capped at the box's per-GPU CPU share ({note})"
    return n, note


def cpu_baseline(args, ms, repeats=3):
    """The CPU restatements on the box's permitted cores, each mode's sample split into `repeats` equal runs
    (the host is shared: one run alone has varied by +-45 % between sessions); value = the median run's rate,
    the spread reported beside it."""
    import oracle
    import rasr_amd as ra
    threads, note = (args.cpu_threads, "--cpu-threads") if args.cpu_threads else available_cpus()
    out = {}
    for name, per_thread in (("SIMD-diagonal-maximum", args.cpu_frames_per_thread),
                             ("diagonal-maximum", max(1, args.cpu_frames_per_thread // 2))):
        n = threads * max(1, per_thread // repeats)
        frames = ra.synthetic_frames(n, args.dim, seed=999)
        o = oracle.OracleSimd(ms) if name.startswith("SIMD") else oracle.OracleFloat(ms)
        rates, total = [], 0.0
        for _ in range(repeats):
            t0 = time.perf_counter()
            o.score(frames, n_threads=threads)
            dt = time.perf_counter() - t0
            rates.append(n / dt)
            total += dt
        rates.sort()
        out[name] = {"value": rates[len(rates) // 2], "frames": n * repeats, "seconds": total,
                     "runs": [round(r, 1) for r in rates]}
        del o
    simd, flt = out["SIMD-diagonal-maximum"], out["diagonal-maximum"]
    return {"value": flt["value"], "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": (f"{flt['frames']} frames x {ms.n_entries} densities in {repeats} runs (median), "
                       f"diagonal-maximum restatement (oracle/gmm_oracle.c orc_float_score, SSE3 distance in the "
                       f"reference's order), {threads} threads, {flt['seconds']:.1f} s; SIMD-diagonal-maximum "
                       f"restatement (SSE2 u8 SSD like the reference JIT): {simd['frames']} frames, "
                       f"{simd['seconds']:.1f} s"),
            "cpu_model": _cpu_model(), "host_logical_cpus": os.cpu_count(), "threads_note": note,
            "runs": {"diagonal-maximum": flt["runs"], "SIMD-diagonal-maximum": simd["runs"]},
            "modes": {"diagonal-maximum": flt["value"], "SIMD-diagonal-maximum": simd["value"]}}


def host_boundary(args, ms, kind, calls=6):
    """gmm_score_host (host frames in, host tables out, PCIe included) into page-locked tables
    (rasr_amd.pinned_empty = gmm_host_alloc), the path an RASR caller reading score(e) on the host takes:
    score + best tables, scores only (GMM_HOST_LAZY_BEST: best densities computed only if fetched later, what the
    search needs and what the C++ drop-in asks for), and scores only frame-major (GMM_HOST_FRAME_MAJOR, the
    drop-in's own table layout)."""
    import rasr_amd as ra
    fpl = args.frames or FRAMES_PER_LAUNCH
    sc = ra.Scorer(ms, kind, max_frames=fpl)
    frames = ra.synthetic_frames(fpl, args.dim, seed=555)
    m = sc.n_mixtures()
    out = ra.pinned_empty((m, fpl), "float32")
    best = ra.pinned_empty((m, fpl), "uint32")
    out_fm = ra.pinned_empty((fpl, m), "float32")
    legs = {
        "scores_and_best": (lambda: sc.score_host(frames, out=out, best_out=best), 8),
        "scores_only": (lambda: sc.score_host_ring(frames, 0, fpl, out, lazy_best=True), 4),
        "scores_only_frame_major": (lambda: sc.score_host_ring(frames, 0, fpl, out_fm, lazy_best=True,
                                                                frame_major=True), 4),
    }
    rec = {"unit": "frames/s", "scorer": kind, "frames_per_call": fpl,
           "path": "gmm_score_host / gmm_score_host_ring into page-locked tables (gmm_host_alloc), PCIe-inclusive; "
                   "not `value`"}
    for name, (fn, bytes_per) in legs.items():
        fn()  # warm-up (pipeline streams, transposed tables)
        t0 = time.perf_counter()
        for _ in range(calls):
            fn()
        dt = time.perf_counter() - t0
        rec[name] = {"value": calls * fpl / dt, "d2h_gb_per_s": calls * fpl * m * bytes_per / dt / 1e9}
    rec["value"] = rec["scores_only"]["value"]
    sc.close()
    return rec


def host_leg_all_ranks(args, ms, kind, ws, rank, local, calls=6):
    """N > 1: the host-buffer path on every rank at once (one process per GPU reading its scores on the host, the
    corpus-partition deployment of src/Bliss/CorpusDescription.cc:167-174): concurrent PCIe and host-memory
    traffic of all ranks.  gmm_score_host_ring, scores only into a page-locked table; barrier-bracketed, the
    slowest rank's time for the aggregate."""
    import rasr_amd as ra
    fpl = args.frames or FRAMES_PER_LAUNCH
    sc = ra.Scorer(ms, kind, max_frames=fpl, device=local)
    frames = ra.synthetic_frames(fpl, args.dim, seed=555 + rank)
    out = ra.pinned_empty((sc.n_mixtures(), fpl), "float32")
    sc.score_host_ring(frames, 0, fpl, out, lazy_best=True)  # warm-up
    barrier(ws)
    t0 = time.perf_counter()
    for _ in range(calls):
        sc.score_host_ring(frames, 0, fpl, out, lazy_best=True)
    dt = time.perf_counter() - t0
    barrier(ws)
    sc.close()
    return host_leg_record(kind, fpl, calls, dt, ws, rank)


def host_leg_record(kind, fpl, calls, dt, ws, rank):
    """Every rank's rate (all-reduce of a one-hot vector) and the aggregate over the slowest rank's time."""
    rates = [calls * fpl / dt]
    dt_max = dt
    if ws > 1:
        import torch
        import torch.distributed as dist
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = torch.zeros(ws + 1, dtype=torch.float64, device=dev)
        t[rank] = calls * fpl / dt
        dist.all_reduce(t)
        m = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        rates, dt_max = [float(x) for x in t[:ws].cpu()], float(m.item())
        backend = "RCCL" if dist.get_backend() == "nccl" else dist.get_backend()
    else:
        backend = None
    return {"scorer": kind, "frames_per_call": fpl, "calls_per_rank": calls, "ranks": ws, "backend": backend,
            "per_rank_frames_per_s": rates, "value": ws * calls * fpl / dt_max, "unit": "frames/s (all ranks)",
            "path": "gmm_score_host_ring, scores only, page-locked table, every rank at once; not `value`"}


def small_batches(args, ms, kind, sizes=(256, 1024, 4096), seconds=0.4):
    """Device-resident scoring at SURVEY 8(d) config 2's batch sizes: frames/s over back-to-back calls of F frames
    (wall clock, launch gaps included) and the scorer kernel's average time and roofline fraction."""
    import torch
    import rasr_amd as ra
    dev = torch.device("cuda", 0)
    out = {}
    for F in sizes:
        sc = ra.Scorer(ms, kind, max_frames=F)
        x = torch.from_numpy(ra.synthetic_frames(F, args.dim, seed=77)).to(dev)
        sres = torch.empty((sc.n_mixtures(), F), dtype=torch.float32, device=dev)
        bres = torch.empty((sc.n_mixtures(), F), dtype=torch.int32, device=dev)
        stream = torch.cuda.current_stream(dev)
        for _ in range(10):
            sc.score_device(x, sres, bres, stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sc.score_device(x, sres, bres, stream)
        torch.cuda.synchronize()
        n = max(20, int(seconds / max(time.perf_counter() - t0, 1e-5)))
        sc.set_timing(True)
        t0 = time.perf_counter()
        for _ in range(n):
            sc.score_device(x, sres, bres, stream)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        kms, nl = sc.kernel_time(reset=True)
        sc.set_timing(False)
        kms /= max(nl, 1)
        kernel = sc.main_kernel()
        peak = PEAK_F16_MFMA_TFLOPS / SPLIT_PRODUCTS if kernel.startswith("scoreSplit") else (
            PEAK_I8_MFMA_TOPS if kernel.startswith("scoreI8") else PEAK_F32_MFMA_TFLOPS)
        frac = 2.0 * args.dim * ms.n_entries * F / (kms * 1e-3) / 1e12 / peak
        out[str(F)] = {"frames_per_s": n * F / dt, "kernel_ms": kms, "kernel": kernel, "roofline_frac": frac,
                       "calls": n}
        del sc, x, sres, bres
        torch.cuda.empty_cache()
    return out


# RASR buffer sizes for the drop-in protocol record and the frames timed at each (about 0.1-0.5 s per size)
DROP_IN_SIZES = [1, 4, 64, 512, 4096, 32768]
DROP_IN_FRAMES = [1500, 6000, 65536, 196608, 262144, 327680]


def drop_in(args, kind):
    """The C++ drop-in (Mm::Gpu::GpuBatchFeatureScorer / GpuFeatureScorer) driven through the recognizer protocol at
    RASR buffer sizes, PCIe and host bookkeeping included: tests/cpp/feature_scorer_driver.cc's bench mode (a child
    process), consuming every emission's score per frame as FeatureScorerNode does; best densities not read (the
    search), plus runs reading them: for every emission (the dump) and for 1-10 emissions per frame (an aligner).
    Reported beside the headline, never `value`."""
    drv = os.path.join(ROOT, "build", "tests", "feature_scorer_driver")
    if not os.access(drv, os.X_OK):
        return {"error": f"{drv} not built"}
    recs = []
    # (sizes, frames, read best densities, share of emissions read per frame in permille): the dump consumer at
    # every size, the aligners' read, and a search-like consumer reading 10 % of the emissions
    # best 2: an aligner's read, bestDensity(e) of 1-10 emissions per frame beside every score (sparse pairs, then
    # best densities carried by every later call)
    runs = [(DROP_IN_SIZES, DROP_IN_FRAMES, 0, 1000), ([4096], [262144], 1, 1000), ([1, 512, 4096], [1500, 196608, 262144], 2, 1000),
            ([512, 4096], [196608, 262144], 0, 100)]
    for sizes, frames, best, permille in runs:
        cmd = [drv, "bench", kind, ",".join(map(str, sizes)), ",".join(map(str, frames)), str(args.mixtures),
               str(args.densities), str(args.dim), str(best), str(permille)]
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        except subprocess.TimeoutExpired:
            return {"error": "driver timed out", "runs": recs}
        if r.returncode != 0:
            return {"error": f"driver exit {r.returncode}: {r.stderr[-300:]}", "runs": recs}
        recs += [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
    return {"scorer": kind, "consumer": "score(e) of every emission per frame (FeatureScorerNode dump); "
                                        "read_permille 100: of a scattered 10 % per frame (the search's active states)",
            "runs": [{k: v for k, v in x.items() if k not in ("mixtures", "densities", "dim", "checksum", "type")}
                     for x in recs]}


def density_sharded_check(args, ms, ws, rank, local, frames_per_call=4096, calls=8):
    """Config 4 on the driver's multi-GPU runs (N > 1, default frame-sharded bench): the density-sharded
    SIMD-diagonal-maximum scorer (rasr_amd.parallel.DensityShardedScorer: 1/N of the densities per rank,
    RCCL all-reduce(MIN) of the split mixtures' packed keys + all-gather) scores one batch on every rank;
    rank 0 compares the assembled table with the unsharded scorer bit for bit (scores and best densities),
    and the path's rate over `calls` calls is reported beside the headline (strong scaling: all ranks score
    the same frames).  Untimed for `value`; any failure is reported in the record, not raised."""
    import torch
    import rasr_amd as ra
    from rasr_amd import parallel
    kind = "SIMD-diagonal-maximum"
    dev = torch.device("cuda", local)
    ds, err = None, None
    try:  # the rank-local part first: a rank that fails here must not leave the others in a collective
        ds = parallel.DensityShardedScorer(ms, kind, frames_per_call, rank, ws, device=local)
    except Exception as e:
        err = f"{type(e).__name__}: {e}"[:300]
    if max_over_ranks(0.0 if ds is not None else 1.0, ws) > 0.0:
        return {"scorer": kind, "error": err or "the density-sharded scorer failed on another rank"}
    try:
        frames = torch.from_numpy(ra.synthetic_frames(frames_per_call, args.dim, seed=4242)).to(dev)
        m_local = ds.scorer.n_mixtures()
        loc_s = torch.empty((m_local, frames_per_call), dtype=torch.float32, device=dev)
        loc_b = torch.empty((m_local, frames_per_call), dtype=torch.int32, device=dev)
        stream = torch.cuda.current_stream(dev)
        full, fullb = ds.score(frames, loc_s, loc_b, stream)
        barrier(ws)
        t0 = time.perf_counter()
        for _ in range(calls):
            ds.score(frames, loc_s, loc_b, stream)
        barrier(ws)
        dt = max_over_ranks(time.perf_counter() - t0, ws)
        import torch.distributed as dist
        coll = "RCCL" if dist.get_backend() == "nccl" else dist.get_backend()
        rec = {"scorer": kind, "layout": f"density-sharded x{ws} + {coll} all-reduce(MIN) of split mixtures + "
                                          f"all-gather", "frames_per_call": frames_per_call,
               "value": calls * frames_per_call / dt, "unit": "frames/s (all ranks score the same frames)"}
        if rank == 0:
            ref = ra.Scorer(ms, kind, max_frames=frames_per_call, device=local)
            rs = torch.empty((ms.n_mixtures, frames_per_call), dtype=torch.float32, device=dev)
            rb = torch.empty((ms.n_mixtures, frames_per_call), dtype=torch.int32, device=dev)
            ref.score_device(frames, rs, rb, stream)
            torch.cuda.synchronize(dev)
            same = bool(torch.equal(full.view(torch.int32), rs.view(torch.int32)) and torch.equal(fullb, rb))
            rec["check"] = "bit-exact vs the unsharded scorer" if same else "MISMATCH vs the unsharded scorer"
            del ref, rs, rb
        del ds, frames, loc_s, loc_b, full, fullb
        torch.cuda.empty_cache()
        return rec
    except Exception as e:  # reported, never fatal to the headline line
        return {"scorer": kind, "error": f"{type(e).__name__}: {e}"[:300]}


CAPI_SHARDED_FRAMES = 4096


def capi_sharded_child(args):
    """One process driving several GPUs, as an RASR process with `density-shard-devices` does:
    gmm_scorer_create_sharded over `--capi-sharded-child` devices (RCCL all-reduce(MIN) exchange when they are
    distinct: ncclCommInitAll + ncclGroupStart/End, one stream per GPU), on the ragged 800k model (K_m ~ U[64,
    256]) whose density boundaries split mixtures, so the reduce really runs.  Checked bit for bit (scores and
    best densities) against the unsharded scorer on device 0; device and host (PCIe-inclusive) calls timed."""
    import numpy as np
    import torch
    import rasr_amd as ra
    devices = [int(d) for d in args.capi_sharded_child.split(",")]
    kind, F, calls = "SIMD-diagonal-maximum", CAPI_SHARDED_FRAMES, 8
    ms = ra.synthetic_mixture_set(args.mixtures, ra.ragged_counts(args.mixtures, args.mixtures * args.densities,
                                                                  seed=99), args.dim, seed=2025)
    frames = ra.synthetic_frames(F, args.dim, seed=4242)
    sh = ra.Scorer(ms, kind, max_frames=F, devices=devices)
    parts, exchange = sh.shard_info()
    dev = torch.device("cuda", devices[0])
    fr = torch.from_numpy(frames).to(dev)
    s = torch.empty((ms.n_mixtures, F), dtype=torch.float32, device=dev)
    b = torch.empty((ms.n_mixtures, F), dtype=torch.int32, device=dev)
    sh.score_device(fr, s, b)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(calls):
        sh.score_device(fr, s, b)
    for d in set(devices):
        torch.cuda.synchronize(torch.device("cuda", d))
    dev_rate = calls * F / (time.perf_counter() - t0)
    hs, hb = sh.score_host(frames)
    t0 = time.perf_counter()
    for _ in range(calls):
        sh.score_host(frames, out=hs, best_out=hb)
    host_rate = calls * F / (time.perf_counter() - t0)
    ref = ra.Scorer(ms, kind, max_frames=F, device=devices[0])
    rs, rb = ref.score_host(frames)
    from rasr_amd import parallel
    split = len(parallel.split_mixtures(parallel.density_shards(ms.mixture_offsets, len(devices))))
    same = (np.array_equal(s.cpu().numpy().view(np.uint32), rs.view(np.uint32)) and
            np.array_equal(b.cpu().numpy().view(np.uint32), rb) and np.array_equal(hs.view(np.uint32), rs.view(np.uint32))
            and np.array_equal(hb, rb))
    return {"scorer": kind, "api": "gmm_scorer_create_sharded (one process, all GPUs)", "devices": devices,
            "parts": parts, "exchange": exchange, "split_mixtures": split, "model": "ragged 800k (K_m ~ U[64, 256])",
            "frames_per_call": F, "device_frames_per_s": dev_rate, "host_frames_per_s": host_rate,
            "check": "bit-exact vs the unsharded scorer" if same else "MISMATCH vs the unsharded scorer"}


# ---------------------------------------------------------------------------
# N > 1: the checks of never-executed multi-GPU paths, fenced in child processes, and the run's deadline
# ---------------------------------------------------------------------------
_DIST_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE",
              "GROUP_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID", "TORCHELASTIC_RESTART_COUNT",
              "TORCHELASTIC_MAX_RESTARTS", "TORCHELASTIC_USE_AGENT_STORE", "TORCH_NCCL_ASYNC_ERROR_HANDLING")


def _kill_session(p) -> None:
    """SIGKILL a fenced child and everything in its session (it was started with start_new_session)."""
    try:
        os.killpg(p.pid, signal.SIGKILL)
    except (ProcessLookupError, PermissionError):
        pass


class LineGuard:
    """The run's JSON line (rank 0), printed exactly once: by `emit()` at the end, or by the deadline watchdog with
    the records that have finished (those still running marked as cut), after which every rank exits -- 0 once the
    headline is measured.  Fenced children still running at the deadline are killed first."""

    def __init__(self, rank: int, deadline_s: float):
        self.rank, self.deadline_s = rank, deadline_s
        self.line = None            # rank 0, once the headline is measured
        self.headline_done = False  # every rank
        self.pending = []           # records started, not finished
        self.children = []          # fenced child processes
        self._lock = threading.Lock()
        self._printed = False
        if deadline_s > 0:
            t = threading.Timer(deadline_s, self._deadline)
            t.daemon = True
            t.start()

    def begin(self, key: str) -> None:
        with self._lock:
            self.pending.append(key)

    def set(self, key: str, value, sub: str | None = None) -> None:
        """line[key] = value (or line[sub][key] = value)."""
        with self._lock:
            if key in self.pending:
                self.pending.remove(key)
            if self.line is not None:
                (self.line[sub] if sub else self.line)[key] = value

    def emit(self) -> None:
        with self._lock:
            if self._printed:
                return
            self._printed = True
            if self.rank == 0 and self.line is not None:
                print(json.dumps(self.line), flush=True)

    def _deadline(self) -> None:
        for p in list(self.children):
            _kill_session(p)
        with self._lock:
            if not self._printed:
                self._printed = True
                if self.rank == 0 and self.line is not None:
                    for k in self.pending:
                        self.line[k] = {"error": f"still running at the {self.deadline_s:.0f} s deadline, cut"}
                    self.line["deadline"] = {"seconds": self.deadline_s, "cut": list(self.pending)}
                    print(json.dumps(self.line), flush=True)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0 if self.headline_done else 3)


def run_fenced(cmds, timeout_s: float, guard: LineGuard, grace_s: float = 10.0) -> dict:
    """Run `cmds` ([(argv, env)], one per rank of a check) as child processes, each in its own session, and return
    the last JSON line rank 0's child printed -- or an error record: the first child that exits non-zero (after
    `grace_s` for the others to fail or finish) or the timeout kills every one of them, since a peer left inside a
    collective would wait forever.  Never raises."""
    procs, errs = [], []
    t0 = time.monotonic()
    try:
        for argv, env in cmds:
            out, err = tempfile.TemporaryFile("w+"), tempfile.TemporaryFile("w+")
            p = subprocess.Popen(argv, env=env, stdout=out, stderr=err, stdin=subprocess.DEVNULL, text=True,
                                 start_new_session=True)
            procs.append((p, out, err))
            guard.children.append(p)
        failed_at, error = None, None
        while True:
            rcs = [p.poll() for p, _, _ in procs]
            if all(rc is not None for rc in rcs):
                break
            now = time.monotonic()
            if failed_at is None and any(rc not in (None, 0) for rc in rcs):
                failed_at = now
            if failed_at is not None and now - failed_at > grace_s:
                break
            if now - t0 > timeout_s:
                alive = [i for i, rc in enumerate(rcs) if rc is None]
                error = f"timed out after {timeout_s:.0f} s (ranks still running: {alive}); killed"
                break
            time.sleep(0.2)
        for p, _, _ in procs:
            if p.poll() is None:
                _kill_session(p)
            p.wait()
        texts = []
        for p, out, err in procs:
            out.seek(0)
            err.seek(0)
            texts.append((p.returncode, out.read(), err.read()))
        bad = [(i, rc, e) for i, (rc, _, e) in enumerate(texts) if rc != 0]
        if error is None and bad:
            i, rc, e = bad[0]
            error = f"rank {i} exited {rc}: {e.strip()[-300:]}"
        if error is None:
            lines = [x for x in texts[0][1].splitlines() if x.startswith("{")]
            if not lines:
                error = "no JSON record from rank 0"
            else:
                rec = json.loads(lines[-1])
                rec["wall_s"] = round(time.monotonic() - t0, 1)
                return rec
        return {"error": error, "wall_s": round(time.monotonic() - t0, 1)}
    except Exception as e:  # never fatal to the line
        for p, _, _ in procs:
            _kill_session(p)
        return {"error": f"{type(e).__name__}: {e}"[:300]}
    finally:
        for p, out, err in procs:
            out.close()
            err.close()
            if p in guard.children:
                guard.children.remove(p)


def density_check_child(args):
    """One rank of the fenced density-sharded check: its own process group (RCCL), the model, the check; rank 0
    prints the record."""
    import torch.distributed as dist
    ws, rank, local = dist_setup(args)
    if fence_probe():
        import torch
        t = torch.ones(1)
        dist.all_reduce(t)
        _inject("raise", rank)
        _inject("hang", rank)
        rec = {"scorer": "probe", "check": "probe", "ranks": ws, "sum": float(t.item())}
    else:
        import rasr_amd as ra
        ms = ra.synthetic_mixture_set(args.mixtures, args.densities, args.dim, seed=2024)
        rec = density_sharded_check(args, ms, ws, rank, local)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    dist.destroy_process_group()


def fenced_extras(args, ws: int, rank: int, guard: LineGuard, group) -> None:
    """Rank 0 runs, one after the other, (1) the density-sharded layout's check over RCCL as N fresh ranks of this
    script (`--density-check-child`: their own process group, so a hang or a failure there cannot take the
    headline's ranks with it) and (2) the C-ABI sharded handle over all GPUs in one child process
    (`--capi-sharded-child`), each killed at FENCE_TIMEOUT_S; the other ranks wait on a gloo barrier.  The
    records (or their errors) go into the line."""
    import torch.distributed as dist
    if rank == 0:
        me = [sys.executable, os.path.abspath(__file__), "--mixtures", str(args.mixtures), "--densities",
              str(args.densities), "--dim", str(args.dim), "--deadline", "0"]
        env0 = {k: v for k, v in os.environ.items() if k not in _DIST_VARS}
        env0.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        port = _free_port()
        cmds = [(me + ["--gpus", str(ws), "--density-check-child"],
                 dict(env0, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(ws), LOCAL_WORLD_SIZE=str(ws),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))) for r in range(ws)]
        guard.begin("density_sharded")
        guard.set("density_sharded", run_fenced(cmds, FENCE_TIMEOUT_S, guard))
        guard.begin("density_sharded_capi")
        if fence_probe():
            n_vis = ws
        else:
            import torch
            n_vis = torch.cuda.device_count()
        if n_vis < ws and os.environ.get("RASR_BENCH_SAME_DEVICE") != "1":
            rec = {"skipped": f"{n_vis} visible devices < {ws} ranks"}
        else:
            devs = ",".join("0" if os.environ.get("RASR_BENCH_SAME_DEVICE") == "1" else str(d) for d in range(ws))
            rec = run_fenced([(me + ["--capi-sharded-child", devs], env0)], FENCE_TIMEOUT_S, guard)
        guard.set("density_sharded_capi", rec)
    dist.barrier(group=group)


def make_line(args, res, ws: int) -> dict:
    n_dens = args.mixtures * args.densities
    return {
        "metric": f"frames/sec scored, {args.dim}-dim x {n_dens // 1000}k-density diag-GMM",
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
            "densities_per_mixture": "U[64, 256] (ragged, same total)" if args.ragged else args.densities,
            "covariance_tying": args.tying,
            "dimension": args.dim,
            "frames_per_gpu_per_step": res["frames_per_step"],
            "frames_per_launch": res["frames_per_launch"],
            "best_density": not (args.no_best or args.mode.startswith("presel") or args.mode == "bint"
                                 or args.mode.endswith("-scores")),
            "parallelism": (f"mixture-sharded x{ws} + RCCL all-gather" if args.parallel == "mixtures" and ws > 1
                            else f"density-sharded x{ws} + RCCL all-reduce(MIN) of split mixtures + all-gather"
                            if args.parallel == "densities" and ws > 1 else f"frame-sharded replicas x{ws}"),
        },
        "timed_region_s": res["timed_region_s"],
        "roofline": res["roofline"],
        "cpu_baseline": None,
        "host_boundary": None,
    }


def main():
    args = parse()
    if args.capi_sharded_child:
        if fence_probe():
            _inject("capi-hang", 0)
            print(json.dumps({"probe": True, "devices": args.capi_sharded_child}), flush=True)
            return
        print(json.dumps(capi_sharded_child(args)), flush=True)
        return
    if args.density_check_child:
        density_check_child(args)
        return
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    if os.environ.get("RASR_BENCH_LAUNCH_PROBE"):  # tests/test_bench_launcher.py: the ranks, no GPU work
        rec = {"rank": int(os.environ.get("RANK", "0")), "world_size": int(os.environ.get("WORLD_SIZE", "1")),
               "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "gpus": args.gpus}
        if os.environ.get("RASR_BENCH_PROBE_HOST_LEG") and rec["world_size"] > 1:
            # the N > 1 host leg's collectives over gloo with a synthetic timing (rank r took (r + 1) / 10 s)
            import torch.distributed as dist
            dist.init_process_group("gloo")
            rec["host_leg"] = host_leg_record("probe", 1000, 3, (rec["rank"] + 1) / 10.0, rec["world_size"],
                                              rec["rank"])
            dist.destroy_process_group()
        with open(os.path.join(os.environ["RASR_BENCH_LAUNCH_PROBE"], f"rank{rec['rank']}.json"), "w") as f:
            json.dump(rec, f)
        return
    probe = fence_probe()
    ws, rank, local = dist_setup(args)
    guard = LineGuard(rank, args.deadline)
    group = None
    if ws > 1:
        import datetime
        import torch.distributed as dist
        # the fenced phase's waiting room: gloo (host), outlasting both fenced children
        group = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=2 * FENCE_TIMEOUT_S + 120))
    launches = args.launches or DEFAULT_LAUNCHES[args.mode]
    if args.mode == "nn" and not probe:
        res = run_nn(args, ws, rank, local, launches)
        guard.headline_done = True
        if rank == 0:
            guard.line = {
                "metric": "frames/sec scored, hybrid-DNN posteriors (Nn::BatchFeatureScorer)", "value": res["value"],
                "unit": "frames/s", "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": res["ms_per_step"], "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                "dtype": res["dtype"], "data": "synthetic (random-init network, frames N(0,1))",
                "config": {"workload": "hybrid DNN " + "-".join(map(str, NN_DIMS)) + f" {args.nn_activation}, 5000 classes",
                           "frames_per_gpu_per_step": res["frames_per_step"],
                           "frames_per_launch": res["frames_per_launch"],
                           "parallelism": f"frame-sharded replicas x{ws}"},
                "timed_region_s": res["timed_region_s"], "roofline": res["roofline"], "cpu_baseline": None}
        guard.emit()
        if ws > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    if probe:  # synthetic headline: the orchestration below is what is under test
        ms = None
        res = {"value": 1.0, "ms_per_step": 1.0, "dtype": "probe", "frames_per_step": 0, "frames_per_launch": 0,
               "timed_region_s": 0.0, "roofline": None}
    else:
        import rasr_amd as ra
        counts = (ra.ragged_counts(args.mixtures, args.mixtures * args.densities) if args.ragged else args.densities)
        ms = ra.synthetic_mixture_set(args.mixtures, counts, args.dim, seed=2024,
                                      tying=None if args.tying == "pooled" else args.tying)
        res = run_mode(args, args.mode, ms, ws, rank, local, launches)
    guard.headline_done = True
    if rank == 0:
        guard.line = make_line(args, res, ws)
    multi = ws > 1 and args.parallel == "frames" and args.mode in ("fp32", "simd")
    if not probe:
        if not args.no_extra_mode:
            # the other headline-model scorers (nn returned above): fp32 / SIMD, and the batched int scorer; the
            # same collectives as the headline
            extra = {}
            for other in [m for m in ("fp32", "simd", "bint", "simd-scores", "fp32-scores") if m != args.mode]:
                r2 = run_mode(args, other, ms, ws, rank, local, DEFAULT_LAUNCHES[other])
                extra[other] = {"value": r2["value"], "ms_per_step": r2["ms_per_step"],
                                "frames_per_gpu_per_step": r2["frames_per_step"],
                                "frames_per_launch": r2["frames_per_launch"], "timed_region_s": r2["timed_region_s"],
                                "dtype": r2["dtype"], "scorer": MODES[other][0], "roofline": r2["roofline"]}
                guard.set("modes", dict(extra))
        if rank == 0 and ws == 1 and args.host_boundary == "auto" and not args.mode.startswith("presel"):
            guard.begin("host_boundary")
            guard.set("host_boundary", host_boundary(args, ms, MODES[args.mode][0]))
        if multi and args.host_boundary == "auto":
            hb_all = host_leg_all_ranks(args, ms, MODES[args.mode][0], ws, rank, local)
            guard.set("host_boundary_all_ranks", hb_all)
            guard.set("process_group", {"backend": hb_all["backend"], "ranks": ws}, sub="config")
        if rank == 0 and ws == 1 and args.extras == "auto" and args.mode in ("fp32", "simd"):
            guard.begin("small_batches")
            guard.set("small_batches", {MODES[m][0]: small_batches(args, ms, MODES[m][0]) for m in ("fp32", "simd")})
            guard.begin("drop_in_protocol")
            guard.set("drop_in_protocol", {MODES[m][0]: drop_in(args, MODES[m][0]) for m in ("fp32", "simd")})
        if rank == 0 and ws == 1 and args.cpu_baseline == "auto":
            guard.begin("cpu_baseline")
            guard.set("cpu_baseline", cpu_baseline(args, ms))
    if multi and not args.no_density_check:
        _inject("parent-hang", rank)
        fenced_extras(args, ws, rank, guard, group)
    guard.emit()
    if ws > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
