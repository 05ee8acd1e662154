#!/usr/bin/env python3
"""How much work could preselection skip on the GPU?  The reference's preselection types (BatchFeatureScorer.cc
238-289, 478-533) score, per frame, only the densities of the n_select clusters nearest to it -- on a CPU that is
the work saved.  A GPU scorer works on (16-density tile) x (16..128-frame block) MFMA products, so it can skip only
a tile none of whose densities any frame of the block selected.  This script measures, with the oracle's
clustering (oracle/oracle.py OraclePresel, the reference's DensityClustering) on the bench's synthetic model and
frames, the union of the clusters selected by a block of frames and the share of skippable (tile, block) pairs.
usage: presel_coverage.py [--mixtures 1250] [--frames 4096]   (test infrastructure: runs the oracle on the CPU)"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mixtures", type=int, default=1250)
    ap.add_argument("--frames", type=int, default=4096)
    a = ap.parse_args()
    import rasr_amd as ra
    from oracle.oracle import OraclePresel
    K = 160
    ms = ra.synthetic_mixture_set(a.mixtures, K, 39, seed=2024)
    op = OraclePresel(ms, "int", clusters=256, select=32)
    sel = op.select(ra.synthetic_frames(a.frames, 39, seed=5))
    cnt = np.bincount(op.cluster_of_entry, minlength=256)
    print(f"clusters selected per frame: {sel.sum(1).mean():.1f} of 256; densities per cluster median "
          f"{np.median(cnt):.0f}")
    tiles = [np.arange(m * K + t0, m * K + t0 + 16) for m in range(a.mixtures) for t0 in range(0, K, 16)]
    for w in (1, 4, 16, 64, 128):
        blocks = sel[: (a.frames // w) * w].reshape(-1, w, 256).max(1)
        covered = (blocks * cnt[None, :]).sum(1).mean() / cnt.sum()
        sample = blocks[:32]
        skip = np.mean([b[op.cluster_of_entry[t]].max() == 0 for b in sample for t in tiles[::7]])
        print(f"block of {w:3d} frames: union {blocks.sum(1).mean():6.1f} clusters, {100 * covered:5.1f} % of the "
              f"densities selected, {100 * skip:5.1f} % of the 16-density tiles skippable")


if __name__ == "__main__":
    main()
