#!/usr/bin/env python3
"""Could diagonal-sum skip work whose contribution underflows?  GaussDiagonalSumFeatureScorer scores a mixture as
best - log sum_d exp(best - s_d) (GaussDiagonalMaximumFeatureScorer.cc:263-289).  A density whose score exceeds the
mixture's best by more than the f32 exp range contributes exactly 0: scoreSplitSum forms 2^(R - kap u) with
v_exp_f32 under flush-to-zero, i.e. 0 once s_d - best > 126 ln 2 = 87.3 (VERDICT r4 item 7 quotes ~104 with
denormals).  A 16-row tile could skip its exponentials only if that held for all 16 rows and every frame of the
wave (64 frames) -- the wave's exp is one instruction for all its lanes.  This script measures, in f64 on the CPU,
on the bench's synthetic model (5000 mixtures x 160 densities, D 39, seed 2024) and on i.i.d. N(0, 1) frames (the
bench) and AR(1) frames (rho 0.95), the distribution of s_d - best per (frame, mixture) and the share of
(tile, 64-frame wave) pairs that are skippable.
usage: sum_underflow.py [--mixtures 500] [--frames 256] [--markdown OUT]   (test infrastructure, CPU only)"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

LIMIT = 126 * np.log(2.0)  # exp(-x) underflows to 0 (FTZ) beyond this


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mixtures", type=int, default=500)
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--markdown", default=None)
    a = ap.parse_args()
    import rasr_amd as ra
    from scripts.presel_coverage import ar1_frames
    ms = ra.synthetic_mixture_set(5000, 160, 39, seed=2024)
    K, D = 160, 39
    var = ms.variances[0].astype(np.float64)
    lognorm = D * np.log(2 * np.pi) + np.log(var).sum()
    means = ms.means[ms.density_mean[ms.mixture_densities[: a.mixtures * K]]].astype(np.float64)  # [M*K, D]
    const = lognorm - 2.0 * ms.mixture_log_weights[: a.mixtures * K]
    lines = [f"model: 5000 x 160 densities (first {a.mixtures} mixtures sampled), D 39; {a.frames} frames; "
             f"limit s_d - best > {LIMIT:.1f}", "",
             "| frames | s_d - best: median | p99 | max | candidates beyond the limit % | skippable (tile, 64-frame wave) % |",
             "|---|---|---|---|---|---|"]
    for name, frames in (("N(0,1) (bench)", ra.synthetic_frames(a.frames, D, seed=5)),
                         ("AR(1) rho 0.95", ar1_frames(a.frames, D, 0.95, 5))):
        x = frames.astype(np.float64) / np.sqrt(var)
        mu = means / np.sqrt(var)
        d2 = (x * x).sum(1)[:, None] - 2 * x @ mu.T + (mu * mu).sum(1)[None, :]
        s = 0.5 * (d2 + const[None, :])                       # [F, M*K]
        s = s.reshape(a.frames, a.mixtures, K)
        gap = s - s.min(axis=2, keepdims=True)
        beyond = gap > LIMIT
        tiles = beyond.reshape(a.frames // 64, 64, a.mixtures, K // 16, 16).all(axis=(1, 4))
        lines.append(f"| {name} | {np.median(gap):.1f} | {np.percentile(gap, 99):.1f} | {gap.max():.1f} | "
                     f"{100 * beyond.mean():.3f} | {100 * tiles.mean():.3f} |")
    print("\n".join(lines))
    if a.markdown:
        with open(a.markdown, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
