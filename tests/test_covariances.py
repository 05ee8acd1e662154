"""Models whose densities do not share one covariance (RASR's covariance-tying = none | mixture-specific-covariance,
src/Mm/Module.cc:54-58, 127-136).  The reference float scorer scores them at the per-density cost of a pooled model
(GaussDiagonalMaximumFeatureScorer.cc:116-218: each density reads its own covariance's 1/sqrt(var) and log-norm).

Float types run the covariance-free split layout (gmm_prepare.cc: one frame operand [(x - c)^2, (x - c)] for every
covariance, K = 6 D + 4, on the split-f16 kernels) -- no per-covariance frame buffers; tolerance 1e-4 relative as the
pooled float path (the near-tie rule for best densities).  The quantized SIMD scorer quantizes the frame per
covariance as the reference's Context does (SimdFeatureScorer.cc:22-35): bit-exact, with a C x frames operand table
whose size is checked at creation (a clear refusal past the device budget)."""
import numpy as np
import pytest

import oracle
import rasr_amd as ra
from test_gpu_parity import _check_float, _assert_bit_exact

TYINGS = ["mixture-specific", "none"]


def test_synthetic_tying():
    ms = ra.synthetic_mixture_set(5, [3, 1, 4, 2, 2], 7, seed=3, tying="mixture-specific")
    assert ms.n_covariances == 5 and list(ms.density_covariance) == [0, 0, 0, 1, 2, 2, 2, 2, 3, 3, 4, 4]
    ms = ra.synthetic_mixture_set(5, 3, 7, seed=3, tying="none")
    assert ms.n_covariances == 15 and np.array_equal(ms.density_covariance, np.arange(15))
    assert ra.synthetic_mixture_set(5, 3, 7, seed=3, tying="pooled").n_covariances == 1


@pytest.mark.gpu
@pytest.mark.parametrize("tying", TYINGS)
@pytest.mark.parametrize("kind", ["diagonal-maximum", "diagonal-sum"])
@pytest.mark.parametrize("d", [39, 16])
def test_float_tying(gpu, tying, kind, d):
    counts = ra.ragged_counts(40, 40 * 12, low=1, high=40, seed=21)
    ms = ra.synthetic_mixture_set(40, counts, d, seed=21, weights="random", tying=tying)
    frames = ra.synthetic_frames(300, d, seed=22)
    sc = ra.Scorer(ms, kind, max_frames=300)
    assert sc.main_kernel() in ("scoreSplit", "scoreSplitWide", "scoreSplitSum")
    s, b = sc.score_host(frames)
    of = oracle.OracleFloatSum(ms) if kind == "diagonal-sum" else oracle.OracleFloat(ms)
    ref_s, ref_b = of.score(frames, n_threads=8)
    _check_float(s, b, ref_s, ref_b, ms, frames, None)


@pytest.mark.gpu
@pytest.mark.parametrize("tying", TYINGS)
def test_float_tying_scales_and_extreme_frames(gpu, tying):
    ms = ra.synthetic_mixture_set(30, 9, 39, seed=23, weights="random", tying=tying)
    frames = ra.synthetic_frames(96, 39, seed=24)
    frames[0] *= 1e12
    frames[1] *= 1e-30
    frames[2] = 0.0
    frames[3, ::2] *= 1e6
    frames[4] *= 3e4
    frames[5, 7] = 1e18
    frames[6:10] *= 40.0
    ref_s, ref_b = oracle.OracleFloat(ms, mixture_weight_scale=0.7, gaussian_scale=1.3).score(frames, 8)
    s, b = ra.Scorer(ms, "diagonal-maximum", max_frames=96, mixture_weight_scale=0.7,
                     gaussian_scale=1.3).score_host(frames)
    _check_float(s, b, ref_s, ref_b, ms, frames, None, mws=0.7, gs=1.3)
    # non-finite frames: the reference's scores (inf / nan) and no best density
    frames2 = ra.synthetic_frames(8, 39, seed=25)
    frames2[0, 3] = np.inf
    frames2[1, 5] = np.nan
    ref_s2, ref_b2 = oracle.OracleFloat(ms).score(frames2)
    s2, b2 = ra.Scorer(ms, "diagonal-maximum", max_frames=8).score_host(frames2)
    assert np.array_equal(np.isnan(s2), np.isnan(ref_s2)) and np.array_equal(np.isinf(s2), np.isinf(ref_s2))
    fin = np.isfinite(ref_s2)
    _check_float(s2[:, 2:], b2[:, 2:], ref_s2[:, 2:], ref_b2[:, 2:], ms, frames2[2:], None)
    assert (b2[:, :2][~fin[:, :2]] == 0xFFFFFFFF).all()


@pytest.mark.gpu
def test_float_tying_offset_narrow(gpu):
    """Per-density covariances on a model far from the origin with narrow variances (|mu / sigma| up to ~200) and
    frames near a density: the expansion about the centre keeps the 1e-4 contract."""
    base = ra.synthetic_mixture_set(40, 12, 39, seed=26, weights="random", tying="none")
    rng = np.random.Generator(np.random.PCG64(27))
    means = base.means.copy()
    means[:, ::2] += np.float32(20.0)
    var = rng.uniform(0.01, 0.1, base.variances.shape).astype(np.float32)
    ms = ra.MixtureSet(means, var, base.density_mean, base.density_covariance, base.mixture_offsets,
                       base.mixture_densities, base.mixture_log_weights)
    dens = rng.integers(0, ms.n_densities, 200)
    sd = np.sqrt(ms.variances[ms.density_covariance[dens]])
    frames = (ms.means[ms.density_mean[dens]] + 0.05 * sd * rng.choice([-1.0, 1.0], size=(200, 39))).astype(np.float32)
    ref_s, ref_b = oracle.OracleFloat(ms).score(frames, n_threads=8)
    s, b = ra.Scorer(ms, "diagonal-maximum", max_frames=200).score_host(frames)
    _check_float(s, b, ref_s, ref_b, ms, frames, None)


@pytest.mark.gpu
def test_float_tying_shards_and_pairs(gpu):
    """Mixture shards and the drop-in's single-pair best densities on a model without tying."""
    ms = ra.synthetic_mixture_set(24, 10, 39, seed=28, weights="random", tying="none")
    frames = ra.synthetic_frames(64, 39, seed=29)
    ref_s, ref_b = oracle.OracleFloat(ms).score(frames, n_threads=8)
    sc = ra.Scorer(ms, "diagonal-maximum", max_frames=64, mixture_range=(5, 17))
    s, b = sc.score_host(frames)
    _check_float(s, b, ref_s[5:17], ref_b[5:17], ms, frames, None, mixture_offset=5)


@pytest.mark.gpu
def test_simd_mixture_specific_bit_exact(gpu):
    ms = ra.synthetic_mixture_set(30, ra.ragged_counts(30, 300, low=1, high=30, seed=30), 39, seed=30,
                                  weights="random", tying="mixture-specific")
    frames = ra.synthetic_frames(200, 39, seed=31)
    ref_s, ref_b, _ = oracle.OracleSimd(ms).score(frames, n_threads=8)
    s, b = ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=200).score_host(frames)
    _assert_bit_exact(s, ref_s)
    assert np.array_equal(b, ref_b)


@pytest.mark.gpu
def test_simd_untied_small_calls_bit_exact_and_refusal(gpu):
    """Untied SIMD: correct at a drop-in buffer size; a per-covariance operand table past the budget is refused
    with a message naming the size (the float types need no such table)."""
    ms = ra.synthetic_mixture_set(20, 8, 39, seed=32, weights="random", tying="none")
    frames = ra.synthetic_frames(16, 39, seed=33)
    ref_s, ref_b, _ = oracle.OracleSimd(ms).score(frames, n_threads=8)
    s, b = ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=16).score_host(frames)
    _assert_bit_exact(s, ref_s)
    assert np.array_equal(b, ref_b)
    big = ra.synthetic_mixture_set(2000, 100, 39, seed=34, tying="none")  # 200k covariances
    with pytest.raises(ra.GmmError, match="covariances"):
        ra.Scorer(big, "SIMD-diagonal-maximum", max_frames=1 << 20)


@pytest.mark.gpu
@pytest.mark.parametrize("tying", TYINGS)
def test_float_tying_density_sharded(gpu, tying):
    """gmm_scorer_create_sharded (three parts on device 0, mixtures split between parts) on a model without a pooled
    covariance: every part on the covariance-free layout, the split mixtures combined by the key exchange."""
    counts = ra.ragged_counts(30, 30 * 14, low=1, high=40, seed=35)
    ms = ra.synthetic_mixture_set(30, counts, 39, seed=35, weights="random", tying=tying)
    frames = ra.synthetic_frames(100, 39, seed=36)
    ref_s, ref_b = oracle.OracleFloat(ms).score(frames, n_threads=8)
    sc = ra.Scorer(ms, "diagonal-maximum", max_frames=128, devices=[0, 0, 0], exchange="copy")
    s, b = sc.score_host(frames)
    _check_float(s, b, ref_s, ref_b, ms, frames, None)


@pytest.mark.gpu
@pytest.mark.parametrize("d,kernel", [(42, "scoreSplit"), (43, "scoreF32"), (20, "scoreSplitWide"), (21, "scoreSplit")])
def test_float_tying_dimension_boundaries(gpu, d, kernel):
    """K = 6 D + 4: the covariance-free layout up to D = 42 (8 K steps; 4 for the 256-frame kernel at D <= 20), the
    f32-MFMA kernel beyond -- the same scores either way."""
    ms = ra.synthetic_mixture_set(12, 9, d, seed=40 + d, weights="random", tying="mixture-specific")
    frames = ra.synthetic_frames(70, d, seed=41)
    sc = ra.Scorer(ms, "diagonal-maximum", max_frames=70)
    assert sc.main_kernel() == kernel
    s, b = sc.score_host(frames)
    ref_s, ref_b = oracle.OracleFloat(ms).score(frames, n_threads=8)
    _check_float(s, b, ref_s, ref_b, ms, frames, None)


@pytest.mark.gpu
def test_sum_tying_edges(gpu):
    """diagonal-sum without tying: an empty mixture (+inf, no density), one-density mixtures (the sum is the
    maximum's score), mixtures past 64 densities, and frames far out."""
    counts = [0, 1, 3, 70, 1, 20]
    ms = ra.synthetic_mixture_set(6, counts, 39, seed=42, weights="random", tying="none")
    frames = ra.synthetic_frames(40, 39, seed=43)
    frames[:4] *= 30.0
    ref_s, ref_b = oracle.OracleFloatSum(ms).score(frames, n_threads=8)
    s, b = ra.Scorer(ms, "diagonal-sum", max_frames=40).score_host(frames)
    assert np.isinf(s[0]).all() and (b[0] == 0xFFFFFFFF).all()
    _check_float(s[1:], b[1:], ref_s[1:], ref_b[1:], ms, frames, None, mixture_offset=1)
