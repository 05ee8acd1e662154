#!/usr/bin/env python3
"""Writes tests/golden/estimator/model.mix (a binary maximum-likelihood estimator file in the layout of
AbstractMixtureSetEstimator::write, src/Mm/AbstractMixtureSetEstimator.cc:481-509) and model_tables.npz (the
mixture set oracle/estimator.py estimates from it with the reference defaults).  The accumulators come from a
Viterbi pass over synthetic frames (two pooled covariances, shared and low-weight densities, an unreferenced
density, one zero-weight mean).  Data only; regenerate with `python scripts/make_estimator_golden.py`."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import estimator as est  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "estimator")


def main():
    rng = np.random.Generator(np.random.PCG64(20240611))
    D, n_dens = 39, 24
    centres = rng.standard_normal((n_dens, D)) * 2
    weights = rng.uniform(0.2, 1.0, n_dens)
    weights[5] = 0.0005   # a low-weight density (removed below minimum-observation-weight 5)
    weights[11] = 0.0     # never observed: its mean has weight 0
    weights[23] = 0.0     # the density no mixture references (its estimators stay empty)
    assign = rng.choice(n_dens, size=4000, p=weights / weights.sum())
    frames = (centres[assign] + rng.standard_normal((4000, D)) * 0.8).astype(np.float32)
    density_mean = np.arange(n_dens)
    density_cov = (np.arange(n_dens) >= 12).astype(np.int64)  # two pooled covariances
    macc, cacc = est.accumulate_viterbi(frames, assign, n_dens, 2, density_mean, density_cov)
    counts = np.bincount(assign, minlength=n_dens).astype(np.float64)
    mixtures = [[(d, counts[d]) for d in range(0, 6)], [(d, counts[d]) for d in range(6, 12) if d != 11] + [(3, counts[3])],
                [(d, counts[d]) for d in range(12, 18)], [(d, counts[d]) for d in range(18, 23)]]  # 23: unused
    dens = [(int(m), int(c)) for m, c in zip(density_mean, density_cov)]
    os.makedirs(OUT, exist_ok=True)
    data = est.write_estimator_file(os.path.join(OUT, "model.mix"), D, macc, cacc, dens, mixtures)
    t = est.estimate(data)
    np.savez_compressed(os.path.join(OUT, "model_tables.npz"), **{k: np.asarray(v) for k, v in t.items()})
    print("wrote", OUT, len(data), "bytes;", len(t["density_mean"]), "densities")


if __name__ == "__main__":
    main()
