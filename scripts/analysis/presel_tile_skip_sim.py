#!/usr/bin/env python3
"""Could preselection skip matrix-core work?  (round-1 VERDICT item 8)

The preselection scorers (BatchFeatureScorer.cc:238-289, 478-533) evaluate, per frame, only the
densities whose DensityClustering cluster is among the frame's `select-clusters` nearest clusters.
On the GPU a wave scores 64 frames against 16-row tiles on the matrix cores, so work can only be
skipped for a tile none of whose clusters ANY of the wave's 64 frames selected.  This simulation
measures that fraction in the most favourable setting we can construct without real speech:

  * a STRUCTURED model: every mixture's densities scattered (sigma_w) around a mixture centre
    (sigma_c), so a mixture covers few clusters (real triphone states are compact like this), and
    each mixture's densities sorted by cluster before tiling (tiles as cluster-pure as they can be);
  * frames in runs of L consecutive frames near one mixture (a phone segment), in time order, and
    also re-sorted by nearest cluster (a frame permutation the scorer could apply per batch);
  * the reference's default clustering: 256 clusters, 32 selected, 5 Lloyd iterations.

Result (profiles/r02/presel_tile_skip_sim.txt): the union of 64 frames' selections covers 212-236 of
the 256 clusters and 90-97 % of the tiles stay active, so skipping cannot make the masked scorer
faster than the unmasked one (which costs the same MFMA work with a cheaper epilogue).
numpy only; ~1 minute.
"""
import numpy as np

rng = np.random.default_rng(1)
M, K, D = 5000, 160, 39          # BASELINE config 2 shape
C, SEL, ITERS = 256, 32, 5       # DensityClustering defaults (DensityClustering.cc:19-32)
SIGMA_C, SIGMA_W = 1.0, 0.35     # spread of mixture centres / of densities around them
F = 8192                         # frames per simulated batch

cen = rng.normal(0, SIGMA_C, (M, D)).astype(np.float32)
means = (cen[:, None, :] + rng.normal(0, SIGMA_W, (M, K, D))).astype(np.float32).reshape(M * K, D)

# Lloyd's k-means over all densities (the reference seeds with rand(); any seeding shows the effect)
cm = means[rng.choice(M * K, C, replace=False)].copy()
mm = (means ** 2).sum(1)
for _ in range(ITERS):
    a = (mm[:, None] - 2 * means @ cm.T + (cm ** 2).sum(1)[None]).argmin(1)
    for c in range(C):
        s = a == c
        if s.any():
            cm[c] = means[s].mean(0)
clu = a.reshape(M, K)
print("clusters per mixture: mean %.1f" % np.mean([len(np.unique(r)) for r in clu]))
tiles = np.sort(clu, 1).reshape(M, K // 16, 16)  # densities sorted by cluster, 16-row tiles


def frame_runs(L):
    out = []
    while len(out) < F:
        m = rng.integers(M)
        for _ in range(L):
            out.append(cen[m] + rng.normal(0, SIGMA_W, D) + rng.normal(0, 0.5, D))
    return np.array(out[:F], np.float32)


for L in (8, 20):
    X = frame_runs(L)
    dist = (X ** 2).sum(1)[:, None] - 2 * X @ cm.T + (cm ** 2).sum(1)[None]
    sel = np.argsort(dist, 1)[:, :SEL]
    selmask = np.zeros((F, C), bool)
    selmask[np.arange(F)[:, None], sel] = True
    for order in ("time", "sorted"):
        S = selmask if order == "time" else selmask[np.argsort(sel[:, 0], kind="stable")]
        U = S.reshape(F // 64, 64, C).any(1)  # union of each wave's selections
        active = np.mean([U[g][tiles].any(2).mean() for g in range(U.shape[0])])
        print("run %d frames, %s order: union %.1f clusters/group, active tiles %.3f"
              % (L, order, U.sum(1).mean(), active))
