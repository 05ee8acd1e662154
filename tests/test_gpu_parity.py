"""GPU parity: the MI355X scorer (through the C-ABI) against the CPU restatement.

Tolerances (written here, per the north star):
  * SIMD-diagonal-maximum, batch-diagonal-maximum-int: BIT-EXACT scores and best densities.
  * diagonal-maximum, batch-diagonal-maximum-float: |gpu - ref| <= 1e-4 * max(1, |ref|); best density
    identical wherever the two best candidates differ by more than that tolerance.  Every float
    kernel is checked: the split-f16 kernel (f32 operands as two f16 pieces) with 32-density tiles
    (v_mfma_f32_32x32x16_f16, the default for mixtures of <= 512 densities) and with 16-density
    tiles (v_mfma_f32_16x16x32_f16, split_tile16=True), and the f32-MFMA kernel (native_f32=True).
"""
import numpy as np
import pytest

import oracle
import rasr_amd as ra

pytestmark = pytest.mark.gpu

REL_TOL = 1e-4
FLOAT_KERNELS = [pytest.param({"split_tile16": True}, id="split16"), pytest.param({"split_tile32": True}, id="split32"),
                 pytest.param({"native_f32": True}, id="native")]
KIND_OPTS = {"": {}, "native": {"native_f32": True}, "split16": {"split_tile16": True},
             "split32": {"split_tile32": True}}


def _gpu_scores(ms, frames, kind, **kw):
    sc = ra.Scorer(ms, kind, max_frames=max(len(frames), 1), **kw)
    return sc.score_host(frames)


def _assert_bit_exact(a, b):
    assert a.shape == b.shape
    diff = np.flatnonzero(a.view(np.uint32).ravel() != b.view(np.uint32).ravel())
    assert diff.size == 0, f"{diff.size} scores differ; first {diff[:5]}: {a.ravel()[diff[:5]]} vs {b.ravel()[diff[:5]]}"


def _assert_close(gpu, ref):
    err = np.abs(gpu.astype(np.float64) - ref.astype(np.float64)) / np.maximum(1.0, np.abs(ref.astype(np.float64)))
    assert err.max() <= REL_TOL, f"max rel err {err.max()}"
    return err


QUANT_CASES = [
    # (mixtures, densities per mixture (int or 'ragged'), dim, covariances, weights, frames)
    (100, 10, 39, 1, "uniform", 1000),
    (37, "ragged", 45, 1, "random", 777),
    (64, 16, 16, 1, "random", 513),
    (20, 33, 39, 3, "random", 300),
    (12, 7, 80, 1, "uniform", 200),
]


def _model(m, k, d, c, w, seed=7):
    if k == "ragged":
        k = ra.ragged_counts(m, m * 20, low=1, high=40, seed=seed)
    return ra.synthetic_mixture_set(m, k, d, seed=seed, n_covariances=c, weights=w)


@pytest.mark.parametrize("case", QUANT_CASES)
def test_simd_diagonal_maximum_bit_exact(gpu, case):
    m, k, d, c, w, f = case
    ms = _model(m, k, d, c, w)
    frames = ra.synthetic_frames(f, d, seed=11)
    ref_s, ref_b, _ = oracle.OracleSimd(ms).score(frames, n_threads=8)
    s, b = _gpu_scores(ms, frames, "SIMD-diagonal-maximum")
    _assert_bit_exact(s, ref_s)
    assert np.array_equal(b, ref_b)


@pytest.mark.parametrize("case", [q for q in QUANT_CASES if q[3] == 1])
def test_batch_int_bit_exact(gpu, case):
    m, k, d, c, w, f = case
    ms = _model(m, k, d, c, w)
    frames = ra.synthetic_frames(f, d, seed=12)
    ref = oracle.batch_int_score(ms, frames, n_threads=8)
    s, _ = _gpu_scores(ms, frames, "batch-diagonal-maximum-int")
    _assert_bit_exact(s, ref)


def _f64_density_score(ms, e, j, x, mws=1.0, gs=1.0):
    """0.5 * (-2 mws log c + gs logNorm + gs * sum((m - x)^2 / var)) in float64 for entry j of mixture e."""
    i = int(ms.mixture_offsets[e]) + int(j)
    d = int(ms.mixture_densities[i])
    var = ms.variances[int(ms.density_covariance[d])].astype(np.float64)
    m = ms.means[int(ms.density_mean[d])].astype(np.float64)
    ln = len(var) * np.log(2 * np.pi) + np.log(var).sum()
    return 0.5 * (-2 * mws * ms.mixture_log_weights[i] + gs * ln + gs * (((m - x) ** 2) / var).sum())


def _check_float(gpu_s, gpu_b, ref_s, ref_b, ms, frames, om, mixture_offset=0, mws=1.0, gs=1.0):
    """Scores within REL_TOL; a different best density is accepted only for a (near) tie: the two
    densities' exact (float64) scores agree within REL_TOL.  Exact ties do occur with duplicated
    densities, where the reference's f32-vs-f64 comparison (GDMFS.cc:131-134) picks by rounding."""
    _assert_close(gpu_s, ref_s)
    if gpu_b is None:
        return
    mism = np.argwhere(gpu_b != ref_b)
    for e, t in mism:
        x = frames[t].astype(np.float64)
        a = _f64_density_score(ms, e + mixture_offset, gpu_b[e, t], x, mws, gs)
        b = _f64_density_score(ms, e + mixture_offset, ref_b[e, t], x, mws, gs)
        assert abs(a - b) <= REL_TOL * max(1.0, abs(b)), f"mixture {e} frame {t}: {gpu_b[e, t]} vs {ref_b[e, t]}"


@pytest.mark.parametrize("kopts", FLOAT_KERNELS)
@pytest.mark.parametrize("case", QUANT_CASES)
def test_diagonal_maximum_fp32(gpu, case, kopts):
    m, k, d, c, w, f = case
    ms = _model(m, k, d, c, w)
    frames = ra.synthetic_frames(f, d, seed=13)
    om = oracle.OracleFloat(ms)
    ref_s, ref_b = om.score(frames, n_threads=8)
    s, b = _gpu_scores(ms, frames, "diagonal-maximum", **kopts)
    _check_float(s, b, ref_s, ref_b, ms, frames, om)


@pytest.mark.parametrize("kopts", FLOAT_KERNELS)
def test_diagonal_maximum_scales(gpu, kopts):
    ms = _model(50, 12, 39, 1, "random")
    frames = ra.synthetic_frames(300, 39, seed=14)
    ref_s, ref_b = oracle.OracleFloat(ms, mixture_weight_scale=0.7, gaussian_scale=1.3).score(frames, 8)
    s, b = _gpu_scores(ms, frames, "diagonal-maximum", mixture_weight_scale=0.7, gaussian_scale=1.3,
                       **kopts)
    _check_float(s, b, ref_s, ref_b, ms, frames, None, mws=0.7, gs=1.3)


@pytest.mark.parametrize("kopts", FLOAT_KERNELS)
@pytest.mark.parametrize("case", [q for q in QUANT_CASES if q[3] == 1])
def test_batch_float_fp32(gpu, case, kopts):
    m, k, d, c, w, f = case
    ms = _model(m, k, d, c, w)
    frames = ra.synthetic_frames(f, d, seed=15)
    ref = oracle.batch_float_score(ms, frames, n_threads=8)
    s, _ = _gpu_scores(ms, frames, "batch-diagonal-maximum-float", **kopts)
    _assert_close(s, ref)


def test_float_kernel_selection(gpu):
    """One covariance -> split-f16 kernel: 32-density tiles where their 16-wide K steps save a step
    (D = 45) and mixtures have <= 512 densities, else 16-density tiles; several covariances or
    GMM_FLAG_NATIVE_F32 -> f32 MFMA."""
    assert ra.Scorer(_model(10, 4, 39, 1, "random"), "diagonal-maximum").main_kernel() == "scoreSplitWide"  # K <= 128
    assert ra.Scorer(_model(10, 4, 39, 1, "random"), "batch-diagonal-maximum-float").main_kernel() == "scoreSplitWide"
    # 32-row tiles where they save > 5 % of K (the 32x32 loop clocks lower): D = 45 (144 vs 160), not D = 39 (128 both)
    assert ra.Scorer(_model(10, 4, 45, 1, "random"), "diagonal-maximum").main_kernel() == "scoreSplit32"
    assert ra.Scorer(_model(10, 4, 9, 1, "random"), "diagonal-maximum").main_kernel() == "scoreSplit32"  # 48 vs 64
    assert ra.Scorer(_model(10, 4, 45, 1, "random"), "diagonal-maximum", split_tile16=True).main_kernel() == "scoreSplit"
    assert ra.Scorer(_model(10, 4, 39, 1, "random"), "diagonal-maximum", split_tile32=True).main_kernel() == "scoreSplit32"
    assert ra.Scorer(_model(4, 600, 45, 1, "random"), "diagonal-maximum").main_kernel() == "scoreSplit"
    assert ra.Scorer(_model(10, 4, 60, 1, "random"), "diagonal-maximum", split_tile32=True).main_kernel() == "scoreSplit"
    # several covariances: the covariance-free split layout (K = 6 D + 4: 8 K steps at D = 39, the pair kernel)
    assert ra.Scorer(_model(10, 4, 39, 3, "random"), "diagonal-maximum").main_kernel() == "scoreSplit"
    assert ra.Scorer(_model(10, 4, 16, 3, "random"), "diagonal-maximum").main_kernel() == "scoreSplitWide"
    assert ra.Scorer(_model(10, 4, 45, 3, "random"), "diagonal-maximum").main_kernel() == "scoreF32"  # 6D+4 > 256
    assert ra.Scorer(_model(10, 4, 39, 1, "random"), "diagonal-maximum", native_f32=True).main_kernel() == "scoreF32"
    assert ra.Scorer(_model(10, 4, 90, 1, "random"), "diagonal-maximum").main_kernel() == "scoreF32"  # 3D+7 > 256


def test_split_accuracy_vs_f32_kernel(gpu):
    """Error of both float kernels against the float64 distance (the oracle accumulates in f64):
    the split-f16 kernel stays in the f32 kernel's accuracy class."""
    ms = _model(200, 24, 39, 1, "random")
    frames = ra.synthetic_frames(1024, 39, seed=31)
    ref_s, _ = oracle.OracleFloat(ms).score(frames, n_threads=8)
    errs = {}
    for name, opts in KIND_OPTS.items():
        s, _ = _gpu_scores(ms, frames, "diagonal-maximum", **opts)
        errs[name] = float((np.abs(s.astype(np.float64) - ref_s) / np.maximum(1.0, np.abs(ref_s))).max())
    print("max rel err split16 %.3g split32 %.3g native %.3g" % (errs["split16"], errs["split32"], errs["native"]))
    for name in ("", "split16", "split32"):  # keys drop <= 8 low mantissa bits: within 2^-17 of the f32 kernel's class
        assert errs[name] <= 1e-5 and errs[name] <= 16 * max(errs["native"], 2.0 ** -22)


@pytest.mark.parametrize("kopts", FLOAT_KERNELS)
def test_float_extreme_frames(gpu, kopts):
    """Per-frame exponent handling: huge, tiny, zero and mixed-magnitude frames."""
    ms = _model(30, 9, 39, 1, "random")
    frames = ra.synthetic_frames(64, 39, seed=32)
    frames[0] *= 1e12
    frames[1] *= 1e-30
    frames[2] = 0.0
    frames[3, ::2] *= 1e6
    frames[4] *= 3e4
    frames[5, 7] = 1e18
    ref_s, ref_b = oracle.OracleFloat(ms).score(frames)
    s, b = _gpu_scores(ms, frames, "diagonal-maximum", **kopts)
    _check_float(s, b, ref_s, ref_b, ms, frames, None)


def _offset_model(m, k, d, c=1, seed=41):
    """Offset, narrow Gaussians: mu ~ N(20, 1) in every other dimension (N(0, 1) in the rest), variances
    U[0.01, 0.1]: |mu / sigma| up to ~200, the regime where the expanded form ||x'||^2 + ||m'||^2 - 2 x'.m'
    of the float kernels cancels (the reference takes (mu - x) isv before squaring,
    GaussDiagonalMaximumFeatureScorer.cc:144-218)."""
    base = _model(m, k, d, c, "random", seed=seed)
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    means = base.means.copy()
    means[:, ::2] += np.float32(20.0)
    var = rng.uniform(0.01, 0.1, (c, d)).astype(np.float32)
    return ra.MixtureSet(means, var, base.density_mean, base.density_covariance, base.mixture_offsets,
                         base.mixture_densities, base.mixture_log_weights)


def _frames_near(ms, n, seed, spread=0.05):
    """Frames at mu_d +- spread * sigma of randomly chosen densities d (the score is then dominated by the
    row constant and a small distance), plus every 8th frame drawn around the model centre."""
    rng = np.random.Generator(np.random.PCG64(seed))
    dens = rng.integers(0, ms.n_densities, n)
    sd = np.sqrt(ms.variances[ms.density_covariance[dens]])
    frames = ms.means[ms.density_mean[dens]] + spread * sd * rng.choice([-1.0, 1.0], size=(n, ms.dimension))
    frames[::8] = ms.means.mean(0) + rng.standard_normal((len(frames[::8]), ms.dimension))
    return frames.astype(np.float32)


@pytest.mark.parametrize("kopts", FLOAT_KERNELS)
@pytest.mark.parametrize("dim", [39, 45])
def test_float_offset_narrow_gaussians(gpu, kopts, dim):
    """Float contract (1e-4 relative) on models far from the origin with narrow variances and frames close
    to a density: the case where an expanded quadratic form about the origin loses ~1e-3."""
    ms = _offset_model(80, "ragged", dim)
    frames = _frames_near(ms, 400, seed=43)
    ref_s, ref_b = oracle.OracleFloat(ms).score(frames, n_threads=8)
    s, b = _gpu_scores(ms, frames, "diagonal-maximum", **kopts)
    _check_float(s, b, ref_s, ref_b, ms, frames, None)
    ref = oracle.batch_float_score(ms, frames, n_threads=8)
    s2, _ = _gpu_scores(ms, frames, "batch-diagonal-maximum-float", **kopts)
    _assert_close(s2, ref)


def test_float_offset_narrow_gaussians_multi_covariance(gpu):
    """Several covariances on the offset, narrow model: the covariance-free split layout (D = 39) and scoreF32
    (||x'||^2 folded into K, native_f32)."""
    ms = _offset_model(40, 12, 39, c=3)
    frames = _frames_near(ms, 300, seed=44)
    ref_s, ref_b = oracle.OracleFloat(ms).score(frames, n_threads=8)
    for opts in ({}, {"native_f32": True}):
        s, b = _gpu_scores(ms, frames, "diagonal-maximum", **opts)
        _check_float(s, b, ref_s, ref_b, ms, frames, None)


def _edge_model():
    """Mixtures with 0, 1, 16, 17 densities, duplicated densities (exact ties), shared densities."""
    rng = np.random.Generator(np.random.PCG64(5))
    d = 39
    n = 60
    means = rng.standard_normal((n, d), dtype=np.float32)
    means[5] = means[4]  # tie inside mixture
    var = (0.5 + np.abs(rng.standard_normal((1, d), dtype=np.float32))).astype(np.float32)
    groups = [[], [0], list(range(1, 17)), list(range(17, 34)), [4, 5, 6], [10, 3, 10, 2], list(range(34, 60))]
    offs = np.cumsum([0] + [len(g) for g in groups]).astype(np.uint32)
    dens = np.array([i for g in groups for i in g], dtype=np.uint32)
    logw = np.concatenate([np.full(len(g), -np.log(max(len(g), 1))) for g in groups])
    return ra.MixtureSet(means, var, np.arange(n, dtype=np.uint32), np.zeros(n, np.uint32), offs, dens, logw)


def test_edge_cases_simd(gpu):
    ms = _edge_model()
    frames = ra.synthetic_frames(130, 39, seed=3)
    frames[0] *= 1000.0   # clipped to 0 / 255 by the quantizer
    frames[1] = 0.0
    frames[2] = ms.means[4]  # exact tie between duplicated densities
    frames[3] = 1e12         # cvttss2si overflow -> 0x80000000 -> quantized 0
    frames[4] = np.nan       # NaN -> 0x80000000 -> quantized 0
    frames[5, ::2] = -np.inf
    ref_s, ref_b, _ = oracle.OracleSimd(ms).score(frames)
    s, b = _gpu_scores(ms, frames, "SIMD-diagonal-maximum")
    _assert_bit_exact(s, ref_s)
    assert np.array_equal(b, ref_b)
    assert b[0, 0] == 0xFFFFFFFF  # empty mixture: bestDensity = (u32)size_t max


@pytest.mark.parametrize("kopts", FLOAT_KERNELS)
def test_edge_cases_float(gpu, kopts):
    ms = _edge_model()
    frames = ra.synthetic_frames(130, 39, seed=4)
    frames[0] *= 1000.0
    frames[2] = ms.means[4]
    ref_s, ref_b = oracle.OracleFloat(ms).score(frames)
    s, b = _gpu_scores(ms, frames, "diagonal-maximum", **kopts)
    assert np.array_equal(s[0], ref_s[0])  # empty mixture: 0.5 * FLT_MAX
    _check_float(s[1:], b[1:], ref_s[1:], ref_b[1:], ms, frames, None, mixture_offset=1)
    assert b[4, 2] == 0  # exact tie between identical rows: the GPU keeps the lowest density index


def test_single_frame_and_strides(gpu):
    import torch
    ms = _model(40, 9, 39, 1, "random")
    frames = ra.synthetic_frames(70, 39, seed=21)
    ref_s, ref_b, _ = oracle.OracleSimd(ms).score(frames)
    sc = ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=70)
    padded = torch.zeros((70, 48), dtype=torch.float32, device=gpu)
    padded[:, :39] = torch.from_numpy(frames).to(gpu)
    out = torch.full((40, 80), -1.0, dtype=torch.float32, device=gpu)
    best = torch.zeros((40, 80), dtype=torch.int32, device=gpu)
    sc.score_device(padded, out, best)
    torch.cuda.synchronize()
    _assert_bit_exact(out[:, :70].cpu().numpy(), ref_s)
    assert np.array_equal(best[:, :70].cpu().numpy().view(np.uint32), ref_b)
    assert (out[:, 70:] == -1).all()
    s1, b1 = sc.score_host(frames[5:6])
    _assert_bit_exact(s1, ref_s[:, 5:6])


def test_score_scale_and_shard(gpu):
    ms = _model(90, 11, 39, 1, "random")
    frames = ra.synthetic_frames(100, 39, seed=22)
    ref_s, ref_b, _ = oracle.OracleSimd(ms).score(frames)
    s, b = _gpu_scores(ms, frames, "SIMD-diagonal-maximum", score_scale=0.25)
    _assert_bit_exact(s, (np.float32(0.25) * ref_s).astype(np.float32))
    # mixture shard [30, 75): same quantization scale as the full model
    sc = ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=100, mixture_range=(30, 75))
    s2, b2 = sc.score_host(frames)
    _assert_bit_exact(s2, ref_s[30:75])
    assert np.array_equal(b2, ref_b[30:75])


def test_quantization_accessors(gpu):
    ms = _model(30, 8, 39, 2, "random")
    o = oracle.OracleSimd(ms)
    sc = ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=4)
    s, q = sc.quantization()
    assert s == o.scaling and q == o.inverse_quantization_factor
    x = ra.synthetic_frames(1, 39, seed=9)[0]
    assert np.array_equal(sc.multiply_and_quantize(x), o.quantize_frame(x))


@pytest.mark.parametrize("dim", [39, 45])
@pytest.mark.parametrize("kind", ["SIMD-diagonal-maximum", "diagonal-maximum", "diagonal-maximum/split32",
                                  "diagonal-maximum/split16", "diagonal-maximum/native"])
def test_full_size_800k_subset(gpu, kind, dim):
    """BASELINE config 2 (5000 x 160 densities, D=39) and config 3 (the same at D=45, LDA+MLLT
    features; default float kernel scoreSplit, scoreSplit32 forced in the split32 case) models: GPU vs oracle on 96 frames."""
    import torch
    ms = ra.synthetic_mixture_set(5000, 160, dim, seed=2024)
    frames = ra.synthetic_frames(96, dim, seed=77)
    kind, _, opt = kind.partition("/")
    if kind == "SIMD-diagonal-maximum":
        ref_s, ref_b, _ = oracle.OracleSimd(ms).score(frames, n_threads=16)
    else:
        ref_s, ref_b = oracle.OracleFloat(ms).score(frames, n_threads=16)
    s, b = _gpu_scores(ms, frames, kind, **KIND_OPTS[opt])
    if kind == "SIMD-diagonal-maximum":
        _assert_bit_exact(s, ref_s)
        assert np.array_equal(b, ref_b)
    else:
        _check_float(s, b, ref_s, ref_b, ms, frames, None)
    del torch


@pytest.mark.parametrize("kind", ["SIMD-diagonal-maximum", "diagonal-maximum", "diagonal-maximum/split32",
                                  "diagonal-maximum/native"])
def test_full_size_batch_invariance(gpu, kind):
    """At the bench size (8192 frames x 800k densities): scoring the whole batch equals scoring
    it in uneven pieces, bit for bit (frames are independent; no cross-frame state)."""
    import torch
    ms = ra.synthetic_mixture_set(5000, 160, 39, seed=2024)
    F = 8192
    frames = torch.from_numpy(ra.synthetic_frames(F, 39, seed=78)).to(gpu)
    kind, _, opt = kind.partition("/")
    sc = ra.Scorer(ms, kind, max_frames=F, **KIND_OPTS[opt])
    M = sc.n_mixtures()
    full = torch.empty((M, F), dtype=torch.float32, device=gpu)
    fullb = torch.empty((M, F), dtype=torch.int32, device=gpu)
    sc.score_device(frames, full, fullb)
    part = torch.empty_like(full)
    partb = torch.empty_like(fullb)
    cuts = [0, 1, 700, 4096, 5000, F]
    for a, b in zip(cuts[:-1], cuts[1:]):
        sc.score_device(frames[a:b], part[:, a:b], partb[:, a:b])
    torch.cuda.synchronize()
    assert torch.equal(full.view(torch.int32), part.view(torch.int32))
    assert torch.equal(fullb, partb)
    assert torch.isfinite(full).all()
    assert int(fullb.min()) >= 0 and int(fullb.max()) < 160


@pytest.mark.parametrize("dim", [39, 45, 33, 48])
def test_batch_fast_bit_exact(gpu, dim):
    """batch-diagonal-maximum-fast (BatchUnrolledIntFeatureScorer, BatchFeatureScorer.cc:558-604) against its
    restatement with the fixed 48-byte loads and mean stride: bit-exact at padded dimension 48."""
    ms = _model(45, "ragged", dim, 1, "random", seed=dim)
    frames = ra.synthetic_frames(300, dim, seed=dim + 1)
    ref = oracle.batch_fast_score(ms, frames)
    s, _ = _gpu_scores(ms, frames, "batch-diagonal-maximum-fast")
    _assert_bit_exact(s, ref)


@pytest.mark.parametrize("dim", [16, 20, 32, 49])
def test_batch_fast_refuses_other_dimensions(gpu, dim):
    """Padded dimension 16 / 32: the reference's unrolled loop reads other rows and past its allocation
    (undefined); > 48: refused by the reference itself (cc:552-555)."""
    ms = _model(5, 4, dim, 1, "random")
    with pytest.raises(ra.GmmError):
        ra.Scorer(ms, "batch-diagonal-maximum-fast", max_frames=8)
