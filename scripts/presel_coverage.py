#!/usr/bin/env python3
"""How much work could preselection skip on the GPU?  The reference's preselection types (BatchFeatureScorer.cc
238-289, 478-533) score, per frame, only the densities of the n_select clusters nearest to it -- on a CPU that is
the work saved.  A GPU scorer works on (16-density tile) x (16..128-frame block) MFMA products, so it can skip only
a tile none of whose densities any frame of the block selected.  This script measures, with the oracle's
clustering (oracle/oracle.py OraclePresel, the reference's DensityClustering) on the bench's synthetic model, the
union of the clusters selected by a block of frames and the share of skippable (tile, block) pairs for three tile
layouts:
  * mixture-major: the scorers' layout, 16 consecutive entries of a mixture per tile;
  * cluster-sorted: a mixture's entries sorted by cluster before tiling (the best a per-mixture layout can do);
  * cluster-major: 16 entries of ONE cluster per tile, across mixtures (the bound: a tile is skippable iff its cluster
    is unselected by the whole block -- but its rows belong to different mixtures, so the per-mixture minimum would
    need a scatter the kernel does not have).
Frames: i.i.d. N(0, 1) (rho 0) as the bench uses, or correlated like speech features, an AR(1) stream per dimension
x_t = rho x_{t-1} + sqrt(1 - rho^2) e_t (stationary N(0, 1), seed recorded).
usage: presel_coverage.py [--mixtures 1250] [--frames 4096] [--rho 0,0.9,0.95,0.97] [--seed 5] [--markdown OUT]
(test infrastructure: runs the oracle on the CPU)"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

BLOCKS = (1, 4, 16, 64, 128)


def ar1_frames(n, d, rho, seed):
    """AR(1) per dimension, stationary N(0, 1): x_0 ~ N(0, 1), x_t = rho x_{t-1} + sqrt(1 - rho^2) e_t."""
    rng = np.random.default_rng(seed)
    e = rng.standard_normal((n, d))
    x = np.empty((n, d))
    x[0] = e[0]
    c = np.sqrt(1.0 - rho * rho)
    for t in range(1, n):
        x[t] = rho * x[t - 1] + c * e[t]
    return x.astype(np.float32)


def skippable(blocks, tile_clusters):
    """Share of (tile, block) pairs with no selected cluster in the tile: blocks [nb, C] bool, tile_clusters a list of
    cluster-index arrays."""
    hit = np.zeros((blocks.shape[0], len(tile_clusters)), bool)
    for j, tc in enumerate(tile_clusters):
        hit[:, j] = blocks[:, tc].any(1)
    return 1.0 - hit.mean()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mixtures", type=int, default=1250)
    ap.add_argument("--frames", type=int, default=4096)
    ap.add_argument("--rho", default="0,0.9,0.95,0.97")
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--markdown", default=None)
    a = ap.parse_args()
    import rasr_amd as ra
    from oracle.oracle import OraclePresel
    K, C = 160, 256
    ms = ra.synthetic_mixture_set(a.mixtures, K, 39, seed=2024)
    op = OraclePresel(ms, "int", clusters=C, select=32)
    coe = np.asarray(op.cluster_of_entry)
    cnt = np.bincount(coe, minlength=C)
    # tile layouts (a sample of every 7th tile for the per-mixture layouts)
    mixture_major = [coe[m * K + t0: m * K + t0 + 16] for m in range(a.mixtures) for t0 in range(0, K, 16)][::7]
    sorted_coe = [np.sort(coe[m * K:(m + 1) * K]) for m in range(a.mixtures)]
    cluster_sorted = [s[t0:t0 + 16] for s in sorted_coe for t0 in range(0, K, 16)][::7]
    # cluster-major: a cluster's entries in tiles of 16 -- the share of tiles skippable is the share of the cluster's
    # tiles, weighted by its tile count
    cl_tiles = (cnt + 15) // 16
    rows = []
    lines = [f"model: {a.mixtures} mixtures x {K} densities, D 39, {C} clusters (select 32), densities per cluster "
             f"median {np.median(cnt):.0f}; {a.frames} frames per stream, seed {a.seed}", ""]
    hdr = ("| rho | clusters/frame | block | union clusters | densities selected % | skippable tiles %: mixture-major "
           "| cluster-sorted | cluster-major (bound) |")
    lines += [hdr, "|---|---|---|---|---|---|---|---|"]
    for rho in [float(r) for r in a.rho.split(",")]:
        frames = ra.synthetic_frames(a.frames, 39, seed=a.seed) if rho == 0 else ar1_frames(a.frames, 39, rho, a.seed)
        sel = op.select(frames).astype(bool)
        per_frame = sel.sum(1).mean()
        for w in BLOCKS:
            blocks = sel[: (a.frames // w) * w].reshape(-1, w, C).any(1)
            covered = (blocks * cnt[None, :]).sum(1).mean() / cnt.sum()
            sample = blocks[:: max(1, blocks.shape[0] // 64)][:64]
            s_mm = skippable(sample, mixture_major)
            s_cs = skippable(sample, cluster_sorted)
            s_cm = 1.0 - (sample * cl_tiles[None, :]).sum(1).mean() / cl_tiles.sum()
            rows.append(dict(rho=rho, w=w, union=float(blocks.sum(1).mean()), covered=float(covered),
                             mixture_major=float(s_mm), cluster_sorted=float(s_cs), cluster_major=float(s_cm)))
            lines.append(f"| {rho:g} | {per_frame:.1f} | {w} | {blocks.sum(1).mean():.1f} | {100 * covered:.1f} | "
                         f"{100 * s_mm:.1f} | {100 * s_cs:.1f} | {100 * s_cm:.1f} |")
    print("\n".join(lines))
    if a.markdown:
        with open(a.markdown, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
