"""diagonal-sum (GaussDiagonalSumFeatureScorer, src/Mm/GaussDiagonalMaximumFeatureScorer.cc:221-298):
score = best - log sum_d exp(best - s_d), best density as diagonal-maximum.

CPU: the oracle restatement against a float64 evaluation of the same formula.
GPU: scoreSplitSum (split-f16 MFMA + online log-sum-exp) against the oracle; tolerance
|gpu - ref| <= 1e-4 * max(1, |ref|) (the f32 contract of the float scorers), best density as in
tests/test_gpu_parity.py (a different one only where the two densities' f64 scores agree).
"""
import numpy as np
import pytest

import oracle
import rasr_amd as ra

REL_TOL = 1e-4


def _f64_sum(ms, frames, mws=1.0, gs=1.0):
    """-log sum_d exp(-s_d) in float64, s_d = 0.5 (-2 mws log c + gs logNorm + gs chi2)."""
    out = np.empty((ms.n_mixtures, len(frames)))
    fr = frames.astype(np.float64)
    for e in range(ms.n_mixtures):
        b, en = int(ms.mixture_offsets[e]), int(ms.mixture_offsets[e + 1])
        if b == en:
            out[e] = np.inf
            continue
        idx = ms.mixture_densities[b:en]
        mean = ms.means[ms.density_mean[idx]].astype(np.float64)            # K x D
        var = ms.variances[ms.density_covariance[idx]].astype(np.float64)   # K x D
        ln = var.shape[1] * np.log(2 * np.pi) + np.log(var).sum(axis=1)
        chi = (((mean[None] - fr[:, None]) ** 2) / var[None]).sum(axis=2)  # F x K
        s = 0.5 * (-2 * mws * ms.mixture_log_weights[b:en][None] + gs * ln[None] + gs * chi)
        best = s.min(axis=1)
        out[e] = best - np.log(np.exp(best[:, None] - s).sum(axis=1))
    return out


def _close(a, ref):
    err = np.abs(a.astype(np.float64) - ref) / np.maximum(1.0, np.abs(ref))
    return float(err.max())


@pytest.mark.parametrize("k", [1, 7, 40])
def test_oracle_sum_vs_float64(k):
    ms = ra.synthetic_mixture_set(12, k, 39, seed=k, weights="random")
    frames = ra.synthetic_frames(20, 39, seed=5)
    s, b = oracle.OracleFloatSum(ms).score(frames, n_threads=2)
    assert _close(s, _f64_sum(ms, frames)) <= 1e-5
    _, bm = oracle.OracleFloat(ms).score(frames, n_threads=2)
    assert np.array_equal(b, bm)  # same best density as diagonal-maximum on these (tie-free) models
    if k == 1:  # one density: the sum is exp(0) = 1, the score is diagonal-maximum's
        sm, _ = oracle.OracleFloat(ms).score(frames)
        assert _close(s, sm.astype(np.float64)) <= 1e-6


def _gpu(ms, frames, **kw):
    sc = ra.Scorer(ms, "diagonal-sum", max_frames=max(len(frames), 1), **kw)
    assert sc.main_kernel() in ("scoreSplitSum", "scoreSplit32Sum")
    return sc.score_host(frames)


def _check(ms, frames, s, b, ref_s, ref_b, mws=1.0, gs=1.0, mixture_offset=0):
    assert _close(s, ref_s.astype(np.float64)) <= REL_TOL
    from test_gpu_parity import _f64_density_score
    for e, t in np.argwhere(b != ref_b):
        x = frames[t].astype(np.float64)
        a1 = _f64_density_score(ms, e + mixture_offset, b[e, t], x, mws, gs)
        a2 = _f64_density_score(ms, e + mixture_offset, ref_b[e, t], x, mws, gs)
        assert abs(a1 - a2) <= REL_TOL * max(1.0, abs(a2)), (e, t, b[e, t], ref_b[e, t])


CASES = [(100, 10, 39, "uniform", 1000), (37, "ragged", 45, "random", 777), (64, 16, 16, "random", 513),
         (12, 7, 80, "uniform", 200), (20, 300, 39, "random", 130)]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_diagonal_sum_gpu(gpu, case):
    m, k, d, w, f = case
    if k == "ragged":
        k = ra.ragged_counts(m, m * 20, low=1, high=40, seed=7)
    ms = ra.synthetic_mixture_set(m, k, d, seed=7, weights=w)
    frames = ra.synthetic_frames(f, d, seed=17)
    ref_s, ref_b = oracle.OracleFloatSum(ms).score(frames, n_threads=8)
    s, b = _gpu(ms, frames)
    _check(ms, frames, s, b, ref_s, ref_b)


@pytest.mark.gpu
def test_diagonal_sum_scales_and_outliers(gpu):
    """mixture-weight-scale / gaussian-scale / score scale, and frames far from every mean (the online
    reference is re-based when a later density is better by more than 2^64)."""
    ms = ra.synthetic_mixture_set(40, 24, 39, seed=8, weights="random")
    frames = ra.synthetic_frames(256, 39, seed=18)
    frames[:32] *= 40.0
    frames[32:40] += 25.0
    ref_s, ref_b = oracle.OracleFloatSum(ms, mixture_weight_scale=0.7, gaussian_scale=1.3).score(frames, 8)
    s, b = _gpu(ms, frames, mixture_weight_scale=0.7, gaussian_scale=1.3)
    _check(ms, frames, s, b, ref_s, ref_b, 0.7, 1.3)
    s2, _ = _gpu(ms, frames, mixture_weight_scale=0.7, gaussian_scale=1.3, score_scale=0.25)
    assert _close(s2, 0.25 * ref_s.astype(np.float64)) <= REL_TOL


@pytest.mark.gpu
def test_diagonal_sum_edges(gpu):
    from test_gpu_parity import _edge_model
    ms = _edge_model()
    frames = ra.synthetic_frames(130, 39, seed=19)
    frames[2] = ms.means[4]
    ref_s, ref_b = oracle.OracleFloatSum(ms).score(frames)
    s, b = _gpu(ms, frames)
    assert np.isinf(s[0]).all() and np.isinf(ref_s[0]).all()  # empty mixture: FLT_MAX - log(0) = +inf
    assert (b[0] == 0xFFFFFFFF).all()
    _check(ms, frames, s[1:], b[1:], ref_s[1:], ref_b[1:], mixture_offset=1)


@pytest.mark.gpu
def test_diagonal_sum_needs_split_kernel(gpu):
    # several covariances: the covariance-free split layout up to dimension 42 (K = 6 D + 4 <= 256), refused beyond
    ms = ra.synthetic_mixture_set(10, 4, 39, seed=1, n_covariances=3)
    assert ra.Scorer(ms, "diagonal-sum").main_kernel() == "scoreSplitSum"
    ms = ra.synthetic_mixture_set(10, 4, 45, seed=1, n_covariances=3)
    with pytest.raises(ra.GmmError, match="diagonal-sum"):
        ra.Scorer(ms, "diagonal-sum")
