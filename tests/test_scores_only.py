"""Calls without best densities (the search's score(e)): the score-only paths.

* SIMD-diagonal-maximum keeps a second copy of its model on the score-only class layout (the `scoresOnly` twin,
  gmm_api.cc; gmm_prepare.cc buildClassLayout): a call with best_density NULL runs scoreI8Seg<SCORE_ONLY> with
  the SIMD constants and finalize.  Its scores must be BIT-EXACT against the oracle (SimdFeatureScorer.cc:135-176)
  and against the key layout, on ragged, tiny and empty mixtures, shards, score scales, strided device frames and
  the quantizer's edge frames.  Models the class layout cannot hold (D > 64, several covariances) keep the key
  layout.
* The float scorers without best densities keep the full f32 value per candidate (no index tag in the low mantissa
  bits): scores within 1e-4 of the oracle as always, and no more than the tag's rounding (2^-16 relative) away
  from the same scorer's scores with best densities.
* GMM_HOST_LAZY_BEST: a host call computes scores only and keeps its frames on the device; gmm_fetch_best_density
  computes the best densities from them when asked (AssigningFeatureScorer.hh:110-121 evaluates bestDensity(e)
  only on request).  They must equal the best densities of a call that asked for them up front.
"""
import numpy as np
import pytest

import oracle
import rasr_amd as ra

pytestmark = pytest.mark.gpu

REL_TOL = 1e-4


def _same(a, b):
    d = np.flatnonzero(a.view(np.uint32).ravel() != b.view(np.uint32).ravel())
    assert d.size == 0, f"{d.size} scores differ; first {d[:5]}: {a.ravel()[d[:5]]} vs {b.ravel()[d[:5]]}"


def _counts(m, k):
    if isinstance(k, tuple) and k[0] == 0:  # empty mixtures included
        return np.random.default_rng(m).integers(0, k[1] + 1, size=m)
    if isinstance(k, tuple):
        return ra.ragged_counts(m, m * (k[0] + k[1]) // 2, low=k[0], high=k[1], seed=m)
    return k


CASES = [
    # mixtures, densities per mixture (int, or (low, high) ragged), dim, covariances, weights, frames
    (60, (1, 40), 39, 1, "random", 301),
    (200, (0, 9), 39, 1, "random", 130),     # empty and tiny mixtures
    (40, 160, 39, 1, "uniform", 257),
    (33, (50, 256), 45, 1, "random", 96),
    (64, 16, 16, 1, "random", 513),
    (25, 3, 64, 1, "random", 77),
    (12, 7, 80, 1, "uniform", 200),           # two K steps: key layout
    (20, 33, 39, 3, "random", 300),           # several covariances: key layout
]


@pytest.mark.parametrize("case", CASES)
def test_simd_scores_only_bit_exact(gpu, case):
    m, k, d, c, w, f = case
    ms = ra.synthetic_mixture_set(m, _counts(m, k), d, seed=23 + m, n_covariances=c, weights=w)
    frames = ra.synthetic_frames(f, d, seed=24)
    ref_s, ref_b, _ = oracle.OracleSimd(ms).score(frames, n_threads=8)
    sc = ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=f)
    s, _ = sc.score_host(frames, want_best=False)
    _same(s, ref_s)
    s2, b2 = sc.score_host(frames)  # the same handle with best densities: the key layout
    _same(s2, ref_s)
    assert np.array_equal(b2, ref_b)
    keys = ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=f, full_keys=True)
    _same(keys.score_host(frames, want_best=False)[0], ref_s)
    # without the score-only twin (GMM_FLAG_NO_SCORE_ONLY_TWIN) every call runs the key layout: same scores
    lone = ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=f, no_score_only_twin=True)
    _same(lone.score_host(frames, want_best=False)[0], ref_s)
    s3, b3 = lone.score_host(frames)
    _same(s3, ref_s)
    assert np.array_equal(b3, ref_b)


def test_simd_scores_only_edge_frames(gpu):
    # mixtures with 0, 1, 16, 17 densities, duplicated densities (exact ties), shared densities
    rng = np.random.Generator(np.random.PCG64(5))
    n = 60
    means = rng.standard_normal((n, 39), dtype=np.float32)
    means[5] = means[4]
    var = (0.5 + np.abs(rng.standard_normal((1, 39), dtype=np.float32))).astype(np.float32)
    groups = [[], [0], list(range(1, 17)), list(range(17, 34)), [4, 5, 6], [10, 3, 10, 2], list(range(34, 60))]
    offs = np.cumsum([0] + [len(g) for g in groups]).astype(np.uint32)
    dens = np.array([i for g in groups for i in g], dtype=np.uint32)
    logw = np.concatenate([np.full(len(g), -np.log(max(len(g), 1))) for g in groups])
    ms = ra.MixtureSet(means, var, np.arange(n, dtype=np.uint32), np.zeros(n, np.uint32), offs, dens, logw)
    frames = ra.synthetic_frames(130, 39, seed=3)
    frames[0] *= 1000.0      # clipped by the quantizer
    frames[1] = 0.0
    frames[2] = ms.means[4]
    frames[3] = 1e12         # cvttss2si overflow
    frames[4] = np.nan
    frames[5, ::2] = -np.inf
    ref_s, _, _ = oracle.OracleSimd(ms).score(frames)
    s, _ = ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=130).score_host(frames, want_best=False)
    _same(s, ref_s)


def test_simd_scores_only_shards_and_scale(gpu):
    ms = ra.synthetic_mixture_set(90, ra.ragged_counts(90, 90 * 30, low=1, high=60, seed=5), 39, seed=6,
                                  weights="random")
    frames = ra.synthetic_frames(200, 39, seed=7)
    ref_s, _, _ = oracle.OracleSimd(ms).score(frames, n_threads=8)
    for lo, hi in ((0, 45), (45, 90), (10, 11)):
        s, _ = ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=200, mixture_range=(lo, hi)).score_host(
            frames, want_best=False)
        _same(s[: hi - lo], ref_s[lo:hi])
    s, _ = ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=200, score_scale=0.75).score_host(frames, want_best=False)
    _same(s, (np.float32(0.75) * ref_s).astype(np.float32))


def test_simd_scores_only_device_strided(gpu):
    import torch
    ms = ra.synthetic_mixture_set(70, ra.ragged_counts(70, 70 * 20, low=1, high=40, seed=9), 39, seed=9,
                                  weights="random")
    frames = ra.synthetic_frames(333, 39, seed=10)
    ref_s, _, _ = oracle.OracleSimd(ms).score(frames, n_threads=8)
    sc = ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=400)
    fr = torch.zeros((333, 48), dtype=torch.float32, device=gpu)
    fr[:, :39] = torch.from_numpy(frames).to(gpu)
    out = torch.full((70, 350), -1.0, dtype=torch.float32, device=gpu)
    sc.score_device(fr, out)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    _same(np.ascontiguousarray(o[:, :333]), ref_s)
    assert (o[:, 333:] == -1.0).all()


FLOAT_KERNELS = [pytest.param({}, id="default"), pytest.param({"split_tile16": True}, id="split16"),
                 pytest.param({"split_tile32": True}, id="split32"), pytest.param({"native_f32": True}, id="native")]


@pytest.mark.parametrize("kind", ["diagonal-maximum", "batch-diagonal-maximum-float"])
@pytest.mark.parametrize("kopts", FLOAT_KERNELS)
@pytest.mark.parametrize("case", [CASES[0], CASES[1], CASES[3], CASES[5]])
def test_float_scores_only(gpu, kind, kopts, case):
    m, k, d, c, w, f = case
    ms = ra.synthetic_mixture_set(m, _counts(m, k), d, seed=31 + m, n_covariances=c, weights=w)
    frames = ra.synthetic_frames(f, d, seed=32)
    if kind == "diagonal-maximum":
        ref = oracle.OracleFloat(ms).score(frames, n_threads=8)[0]
    else:
        ref = oracle.batch_float_score(ms, frames, n_threads=8)
    sc = ra.Scorer(ms, kind, max_frames=f, **kopts)
    s, _ = sc.score_host(frames, want_best=False)
    r64 = ref.astype(np.float64)
    fin = np.abs(r64) < 1e30  # empty mixtures: the type's "no score" value, compared exactly
    assert np.array_equal(s[~fin], ref[~fin])
    err = np.abs(s.astype(np.float64) - r64)[fin] / np.maximum(1.0, np.abs(r64[fin]))
    assert err.max() <= REL_TOL, f"max rel err {err.max()}"
    if kind == "diagonal-maximum":
        # the keyed scores (best densities asked for) differ by at most the tag's rounding
        sk, _ = sc.score_host(frames)
        rel = np.abs(sk.astype(np.float64) - s)[fin] / np.abs(s[fin]).astype(np.float64).clip(1e-30)
        assert rel.max() <= 2.0 ** -15, f"keyed vs untagged {rel.max()}"


@pytest.mark.parametrize("kind", ["SIMD-diagonal-maximum", "diagonal-maximum"])
@pytest.mark.parametrize("frame_major", [False, True])
def test_lazy_best_host(gpu, kind, frame_major):
    ms = ra.synthetic_mixture_set(80, ra.ragged_counts(80, 80 * 25, low=1, high=50, seed=41), 39, seed=41,
                                  weights="random")
    R = 96
    ring = ra.synthetic_frames(R, 39, seed=42)
    sc = ra.Scorer(ms, kind, max_frames=R)
    m = sc.n_mixtures()
    shape = (R, m) if frame_major else (m, R)
    first, n = 70, 60  # wraps
    eager_s, eager_b = np.zeros(shape, np.float32), np.zeros(shape, np.uint32)
    sc.score_host_ring(ring, first, n, eager_s, eager_b, frame_major=frame_major)
    lazy_s, lazy_b = np.zeros(shape, np.float32), np.zeros(shape, np.uint32)
    cid = sc.score_host_ring(ring, first, n, lazy_s, lazy_best=True, frame_major=frame_major)
    plain, _ = sc.score_host(ring[(first + np.arange(n)) % R], want_best=False)  # scores-only, unwrapped
    pos = (first + np.arange(n)) % R
    got = lazy_s[pos] if frame_major else lazy_s[:, pos].T
    _same(np.ascontiguousarray(got), np.ascontiguousarray(plain.T))
    # score_host above replaced the kept frames: the fetch is refused, the caller scores again
    with pytest.raises(ra.GmmError):
        sc.fetch_best(cid, lazy_b)
    cid = sc.score_host_ring(ring, first, n, lazy_s, lazy_best=True, frame_major=frame_major)
    sc.fetch_best(cid, lazy_b)
    sc.fetch_best(cid, lazy_b)  # computed once, copied again
    sel = (lambda t: t[pos]) if frame_major else (lambda t: t[:, pos])
    assert np.array_equal(sel(lazy_b), sel(eager_b))
    if kind == "SIMD-diagonal-maximum":
        _same(np.ascontiguousarray(sel(lazy_s)), np.ascontiguousarray(sel(eager_s)))


def test_lazy_best_batch_type_and_flags(gpu):
    ms = ra.synthetic_mixture_set(20, 8, 39, seed=1)
    frames = ra.synthetic_frames(32, 39, seed=2)
    sc = ra.Scorer(ms, "batch-diagonal-maximum-int", max_frames=32)
    out = np.zeros((20, 32), np.float32)
    cid = sc.score_host_ring(frames, 0, 32, out, lazy_best=True)  # batch types: nothing to keep
    _same(out, oracle.batch_int_score(ms, frames))
    with pytest.raises(ra.GmmError):
        sc.fetch_best(cid, np.zeros((20, 32), np.uint32))
    simd = ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=32)
    with pytest.raises(ra.GmmError):
        simd.score_host_ring(frames, 0, 32, out, keep_best=True, lazy_best=True)
    with pytest.raises(ra.GmmError):
        simd.score_host_ring(frames, 0, 32, out, np.zeros((20, 32), np.uint32), lazy_best=True)


@pytest.mark.parametrize("case", [CASES[0], CASES[1], CASES[2], CASES[3]])
def test_diagonal_sum_scores_only(gpu, case):
    """diagonal-sum without best densities: the running minimum (for the log-sum-exp re-base only) on untagged
    values; the scores as with best densities, within the float contract of the oracle."""
    m, k, d, c, w, f = case
    ms = ra.synthetic_mixture_set(m, _counts(m, k), d, seed=51 + m, n_covariances=c, weights=w)
    frames = ra.synthetic_frames(f, d, seed=52)
    ref = oracle.OracleFloatSum(ms).score(frames, n_threads=8)[0]
    sc = ra.Scorer(ms, "diagonal-sum", max_frames=f)
    s, _ = sc.score_host(frames, want_best=False)
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(s), fin)
    # empty mixtures: the non-finite value itself (NaN or the sign of an infinity) must match, exactly
    assert np.array_equal(s[~fin], ref[~fin], equal_nan=True), f"non-finite {s[~fin][:5]} vs {ref[~fin][:5]}"
    r64 = ref[fin].astype(np.float64)  # masked before subtracting: no inf - inf
    err = np.abs(s[fin].astype(np.float64) - r64) / np.maximum(1.0, np.abs(r64))
    assert err.max() <= REL_TOL, f"max rel err {err.max()}"
    sk, _ = sc.score_host(frames)
    assert np.array_equal(sk[~fin], s[~fin], equal_nan=True)
    s64 = s[fin].astype(np.float64)
    err2 = np.abs(sk[fin].astype(np.float64) - s64) / np.maximum(1.0, np.abs(s64))
    assert err2.max() <= 1e-5, f"with vs without best densities {err2.max()}"
