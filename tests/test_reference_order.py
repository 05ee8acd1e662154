"""Reference-order float scorers (GMM_FLAG_REFERENCE_ORDER, rasr_amd/csrc/gmm_kernels_direct.hip): every
density evaluated in the reference's own f32 operation order, so scores and best densities are BIT-EXACT
against the CPU restatement compiled with the reference's flags (oracle/gmm_oracle.c: orc_float_score for
diagonal-maximum, GaussDiagonalMaximumFeatureScorer.cc:116-181; orc_batch_float_score for
batch-diagonal-maximum-float, BatchFeatureScorer.cc:187-234) -- including near ties, which the matrix-core
kernels resolve only within the float contract."""
import numpy as np
import pytest

import oracle
import rasr_amd as ra

pytestmark = pytest.mark.gpu

CASES = [
    # (mixtures, densities per mixture (int or 'ragged'), dim, covariances, weights, frames)
    (100, 10, 39, 1, "uniform", 700),
    (37, "ragged", 45, 1, "random", 333),
    (64, 16, 16, 1, "random", 300),
    (20, 33, 39, 3, "random", 300),
    (12, 7, 80, 1, "uniform", 200),
    (9, 5, 3, 1, "random", 130),     # D < 4: only the remaining-terms path
    (9, 5, 4, 2, "random", 130),     # D % 4 == 0: no remaining terms
    (6, 4, 128, 1, "random", 70),    # the largest supported dimension
]


def _model(m, k, d, c, w, seed=7):
    if k == "ragged":
        k = ra.ragged_counts(m, m * 20, low=1, high=40, seed=seed)
    return ra.synthetic_mixture_set(m, k, d, seed=seed, n_covariances=c, weights=w)


def _same(a, b):
    assert a.shape == b.shape
    diff = np.flatnonzero(a.view(np.uint32).ravel() != b.view(np.uint32).ravel())
    assert diff.size == 0, f"{diff.size} differ; first {diff[:5]}: {a.ravel()[diff[:5]]} vs {b.ravel()[diff[:5]]}"


@pytest.mark.parametrize("case", CASES, ids=[f"D{c[2]}C{c[3]}" for c in CASES])
def test_diagonal_maximum_bit_exact(gpu, case):
    m, k, d, c, w, f = case
    ms = _model(m, k, d, c, w)
    frames = ra.synthetic_frames(f, d, seed=21)
    ref_s, ref_b = oracle.OracleFloat(ms).score(frames, n_threads=8)
    sc = ra.Scorer(ms, "diagonal-maximum", max_frames=f, reference_order=True)
    assert sc.main_kernel() == "scoreDirect"
    s, b = sc.score_host(frames)
    _same(s, ref_s)
    assert np.array_equal(b, ref_b)


@pytest.mark.parametrize("case", [c for c in CASES if c[3] == 1], ids=[f"D{c[2]}" for c in CASES if c[3] == 1])
def test_batch_float_bit_exact(gpu, case):
    m, k, d, c, w, f = case
    ms = _model(m, k, d, c, w)
    frames = ra.synthetic_frames(f, d, seed=22)
    ref = oracle.batch_float_score(ms, frames, n_threads=8)
    s, _ = ra.Scorer(ms, "batch-diagonal-maximum-float", max_frames=f, reference_order=True).score_host(frames)
    _same(s, ref)


def test_scales_shards_and_edges(gpu):
    """mixture-weight-scale / gaussian-scale / acoustic scale, a mixture shard, and the edge model
    (empty mixture, duplicated densities = exact ties, NaN / inf / huge features)."""
    ms = _model(30, "ragged", 39, 1, "random", seed=3)
    frames = ra.synthetic_frames(257, 39, seed=23)
    frames[3] = np.nan
    frames[4, 5] = np.inf
    frames[5] *= 1e12
    ref_s, ref_b = oracle.OracleFloat(ms, mixture_weight_scale=0.7, gaussian_scale=1.3).score(frames, n_threads=8)
    sc = ra.Scorer(ms, "diagonal-maximum", max_frames=300, reference_order=True, mixture_weight_scale=0.7,
                   gaussian_scale=1.3, score_scale=1.0)
    s, b = sc.score_host(frames)
    _same(s, ref_s)
    assert np.array_equal(b, ref_b)
    # acoustic scale: ScaledContextScorer multiplies the f32 score
    s2, _ = ra.Scorer(ms, "diagonal-maximum", max_frames=300, reference_order=True, mixture_weight_scale=0.7,
                      gaussian_scale=1.3, score_scale=0.25).score_host(frames)
    _same(s2, (np.float32(0.25) * ref_s).astype(np.float32))
    # a mixture shard scores its rows of the table
    s3, b3 = ra.Scorer(ms, "diagonal-maximum", max_frames=300, reference_order=True, mixture_weight_scale=0.7,
                       gaussian_scale=1.3, mixture_range=(7, 19)).score_host(frames)
    _same(s3, ref_s[7:19])
    assert np.array_equal(b3, ref_b[7:19])


def test_edge_model_ties(gpu):
    rng = np.random.Generator(np.random.PCG64(5))
    d, n = 39, 60
    means = rng.standard_normal((n, d), dtype=np.float32)
    means[5] = means[4]
    var = (0.5 + np.abs(rng.standard_normal((1, d), dtype=np.float32))).astype(np.float32)
    groups = [[], [0], list(range(1, 17)), list(range(17, 34)), [4, 5, 6], [10, 3, 10, 2], list(range(34, 60))]
    offs = np.cumsum([0] + [len(g) for g in groups]).astype(np.uint32)
    dens = np.array([i for g in groups for i in g], dtype=np.uint32)
    logw = np.concatenate([np.full(len(g), -np.log(max(len(g), 1))) for g in groups])
    ms = ra.MixtureSet(means, var, np.arange(n, dtype=np.uint32), np.zeros(n, np.uint32), offs, dens, logw)
    frames = np.concatenate([means[[4, 10, 2]], ra.synthetic_frames(61, d, seed=24)]).astype(np.float32)
    ref_s, ref_b = oracle.OracleFloat(ms).score(frames, n_threads=4)
    s, b = ra.Scorer(ms, "diagonal-maximum", max_frames=64, reference_order=True).score_host(frames)
    _same(s, ref_s)
    assert np.array_equal(b, ref_b)
    ref = oracle.batch_float_score(ms, frames, n_threads=4)
    s2, _ = ra.Scorer(ms, "batch-diagonal-maximum-float", max_frames=64, reference_order=True).score_host(frames)
    _same(s2, ref)


@pytest.mark.parametrize("dim", [39, 45])
def test_full_size_800k_bit_exact(gpu, dim):
    """BASELINE configs 2 / 3 model (5000 x 160 densities) on 64 frames: bit-exact scores and densities."""
    ms = ra.synthetic_mixture_set(5000, 160, dim, seed=2024)
    frames = ra.synthetic_frames(64, dim, seed=81)
    ref_s, ref_b = oracle.OracleFloat(ms).score(frames, n_threads=16)
    s, b = ra.Scorer(ms, "diagonal-maximum", max_frames=64, reference_order=True).score_host(frames)
    _same(s, ref_s)
    assert np.array_equal(b, ref_b)


def test_refused_for_other_types(gpu):
    ms = _model(5, 4, 39, 1, "random")
    for kind in ("SIMD-diagonal-maximum", "diagonal-sum", "preselection-batch-float", "batch-diagonal-maximum-int"):
        with pytest.raises(ra.GmmError):
            ra.Scorer(ms, kind, max_frames=8, reference_order=True)
    with pytest.raises(ra.GmmError):  # dimension > 128
        ra.Scorer(_model(3, 2, 130, 1, "random"), "diagonal-maximum", max_frames=8, reference_order=True)
