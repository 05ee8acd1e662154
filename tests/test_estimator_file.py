"""Binary maximum-likelihood estimator files (the reference's default mixture-set reader for every name other than
".pms"/".gz", src/Mm/MixtureSetReader.hh:105-117, MixtureSetReader.cc:52-74): the library's reader
(rasr_amd/csrc/host/MixtureSetEstimatorFile.cc) against oracle/estimator.py's restatement of read + estimate
(AbstractMixtureSetEstimator.cc:299-337, 433-479) on files written in the reference's layout, bit for bit; the
golden fixture; the reference's failure cases; a Viterbi-trained model whose estimate equals the sample moments.
"""
import os

import numpy as np
import pytest

import rasr_amd as ra
from oracle import estimator as est

HERE = os.path.dirname(os.path.abspath(__file__))
FIELDS = ["means", "variances", "density_mean", "density_covariance", "mixture_offsets", "mixture_densities",
          "mixture_log_weights"]


def _same(ms, ref):
    assert ms.dimension == ref["dimension"]
    for f in FIELDS:
        a, b = np.asarray(getattr(ms, f)), np.asarray(ref[f])
        assert a.shape == b.shape, f
        assert np.array_equal(a.view(np.uint8), b.astype(a.dtype).view(np.uint8)), f


def _random_file(seed, D=7, n_means=12, n_covs=3, n_dens=14, n_mix=5, version=2, unused=True):
    rng = np.random.Generator(np.random.PCG64(seed))
    means = []
    for i in range(n_means):
        w = float(rng.integers(0, 40)) if version == 0 else float(rng.uniform(0, 40))
        if i % 5 == 3:
            w = 0.0  # zero-weight mean: estimate() gives a zero mean
        means.append((rng.standard_normal(D) * 3 * max(w, 1), w))
    dens = [(int(rng.integers(0, n_means)), int(rng.integers(0, n_covs))) for _ in range(n_dens)]
    mixtures = []
    for m in range(n_mix):
        k = int(rng.integers(1, 6))
        ids = rng.choice(n_dens - (2 if unused else 0), size=k, replace=False)  # the last two may stay unused
        mixtures.append([(int(d), float(rng.integers(1, 60)) if version == 0 else float(rng.uniform(0.5, 60)))
                         for d in ids])
    # covariance accumulators consistent with their means (weights equal, sums of squares above the mean terms)
    covs = []
    for c in range(n_covs):
        ms_ = sorted({m for mix in mixtures for d, _ in mix for m in [dens[d][0]] if dens[d][1] == c})
        w = sum(means[m][1] for m in ms_ if means[m][1] > 0)
        sq = np.zeros(D)
        for m in ms_:
            s, mw = means[m]
            if mw > 0:
                sq += s * s / mw + mw * rng.uniform(0.2, 2.0, D)
        covs.append((sq, w))
    return est.write_estimator_file(None, D, means, covs, dens, mixtures, version=version)


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("version", [2, 0])
def test_reader_matches_restatement(seed, version):
    data = _random_file(seed, version=version)
    try:
        ref = est.estimate(data)
    except est.EstimatorError:
        with pytest.raises(ra.GmmError):
            ra.estimate_mixture_set(data)
        return
    _same(ra.estimate_mixture_set(data), ref)


@pytest.mark.parametrize("kw", [dict(minimum_observation_weight=0.0), dict(minimum_observation_weight=20.0),
                                dict(minimum_relative_weight=0.3), dict(minimum_variance=0.75),
                                dict(normalize_mixture_weights=False),
                                dict(allow_zero_weights=True, minimum_observation_weight=1.0)])
def test_estimation_parameters(kw):
    for seed in range(6):
        data = _random_file(100 + seed)
        try:
            ref = est.estimate(data, **kw)
        except est.EstimatorError:
            with pytest.raises(ra.GmmError):
                ra.estimate_mixture_set(data, **kw)
            continue
        _same(ra.estimate_mixture_set(data, **kw), ref)


def test_read_dispatch_by_extension(tmp_path):
    """MixtureSetReader: ".pms"/".gz" -> text format, any other extension (or none) -> estimator file."""
    data = _random_file(7)
    ref = est.estimate(data)
    for name in ["model.mix", "model.acc", "model", "dir.v1/model"]:
        p = tmp_path / name
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_bytes(data)
        _same(ra.read_mixture_set(str(p)), ref)
    # the same bytes under a text-format name are parsed as text and refused
    p = tmp_path / "model.pms"
    p.write_bytes(data)
    with pytest.raises(ra.GmmError):
        ra.read_mixture_set(str(p))


def test_offset_and_reduced_dimension(tmp_path):
    """Module_::readMixtureSet applies the dimension offset / reduction to the estimated set as to a text one."""
    data = _random_file(8, D=9)
    ref = est.estimate(data)
    p = tmp_path / "m.mix"
    p.write_bytes(data)
    ms = ra.read_mixture_set(str(p), 2, 0)
    assert np.array_equal(ms.means, ref["means"][:, 2:]) and np.array_equal(ms.variances, ref["variances"][:, 2:])
    ms = ra.read_mixture_set(str(p), 1, 10)
    assert ms.dimension == 10
    assert np.array_equal(ms.means[:, :8], ref["means"][:, 1:]) and (ms.means[:, 8:] == 0).all()
    assert np.array_equal(ms.variances[:, :8], ref["variances"][:, 1:]) and (ms.variances[:, 8:] == 1).all()


def _tiny():
    D = 3
    means = [(np.array([2.0, 4.0, 6.0]), 2.0), (np.array([-3.0, 3.0, 0.0]), 3.0)]
    covs = [(np.array([7.0, 12.0, 21.0]), 5.0)]  # = the mean terms [5, 11, 18] + 5 * [0.4, 0.2, 0.6]
    dens = [(0, 0), (1, 0)]
    mixtures = [[(0, 2.0), (1, 3.0)]]
    return D, means, covs, dens, mixtures


def test_known_answer():
    """Hand-derived: means = sums / weights, variance = (sum x^2 - sum_m s_m^2 / w_m) / w, log weights normalized."""
    D, means, covs, dens, mixtures = _tiny()
    ms = ra.estimate_mixture_set(est.write_estimator_file(None, D, means, covs, dens, mixtures),
                                 minimum_observation_weight=0.0)
    assert np.array_equal(ms.means, np.array([[1, 2, 3], [-1, 1, 0]], np.float32))
    # wmss = [4/2 + 9/3, 16/2 + 9/3, 36/2 + 0] = [5, 11, 18]; sums [7, 12, 21] -> ([2, 1, 3]) / 5
    assert np.array_equal(ms.variances, np.array([[0.4, 0.2, 0.6]], np.float32))
    assert np.allclose(ms.mixture_log_weights, np.log([0.4, 0.6]), rtol=0, atol=1e-15)


@pytest.mark.parametrize("case", ["magic", "truncated", "density_index", "mixture_index", "zero_weight_mixture",
                                  "empty_mixture", "covariance_weight", "negative_covariance_weight", "size"])
def test_reference_failures(case):
    D, means, covs, dens, mixtures = _tiny()
    if case == "density_index":
        dens = [(0, 0), (5, 0)]
    elif case == "mixture_index":
        mixtures = [[(0, 2.0), (9, 3.0)]]
    elif case == "zero_weight_mixture":
        mixtures = [[(0, 2.0), (1, 3.0)], [(1, 0.0)]]
    elif case == "empty_mixture":
        mixtures = [[(0, 2.0), (1, 3.0)], []]
    elif case == "covariance_weight":
        covs = [(covs[0][0], 7.0)]
    elif case == "negative_covariance_weight":  # verify(accumulator_.weight() > 0), GaussDensityEstimator.cc:216
        covs = [(covs[0][0], -5.0)]
    elif case == "size":
        means = [(np.array([2.0, 4.0]), 2.0), means[1]]
    data = est.write_estimator_file(None, D, means, covs, dens, mixtures)
    if case == "magic":
        data = b"MIXSEX\0\0" + data[8:]
    elif case == "truncated":
        data = data[:-5]
    with pytest.raises(est.EstimatorError):
        est.estimate(data, minimum_observation_weight=0.0)
    with pytest.raises(ra.GmmError):
        ra.estimate_mixture_set(data, minimum_observation_weight=0.0)


def test_viterbi_trained_model():
    """A model trained by Viterbi accumulation (each frame counted in its density's mean estimator and its
    covariance's estimator) is estimated to the sample moments of the frames."""
    rng = np.random.Generator(np.random.PCG64(3))
    D, n_dens = 6, 10
    true_means = rng.standard_normal((n_dens, D)) * 4
    assign = rng.integers(0, n_dens, 3000)
    frames = (true_means[assign] + rng.standard_normal((3000, D)) * 0.7).astype(np.float32)
    dm, dc = np.arange(n_dens), np.zeros(n_dens, np.int64)
    macc, cacc = est.accumulate_viterbi(frames, assign, n_dens, 1, dm, dc)
    counts = np.bincount(assign, minlength=n_dens).astype(float)
    mixtures = [[(0, counts[0]), (1, counts[1]), (2, counts[2])], [(d, counts[d]) for d in range(3, n_dens)]]
    data = est.write_estimator_file(None, D, macc, cacc, [(int(m), int(c)) for m, c in zip(dm, dc)], mixtures)
    ms = ra.estimate_mixture_set(data)
    _same(ms, est.estimate(data))
    f64 = frames.astype(np.float64)
    sample_means = np.stack([f64[assign == d].mean(0) for d in range(n_dens)])
    assert np.allclose(ms.means, sample_means, rtol=1e-6, atol=1e-6)
    pooled = sum(((f64[assign == d] - sample_means[d]) ** 2).sum(0) for d in range(n_dens)) / len(frames)
    assert np.allclose(ms.variances[0], pooled, rtol=1e-4)
    w0 = counts[:3] / counts[:3].sum()
    assert np.allclose(np.exp(ms.mixture_log_weights[:3]), w0, rtol=1e-12)


def test_golden_estimator_file():
    """tests/golden/estimator/model.mix (scripts/make_estimator_golden.py) -> the frozen tables, bit for bit."""
    src = os.path.join(HERE, "golden", "estimator", "model.mix")
    ref = np.load(os.path.join(HERE, "golden", "estimator", "model_tables.npz"), allow_pickle=False)
    ms = ra.read_mixture_set(src)
    assert ms.dimension == int(ref["dimension"])
    for f in FIELDS:
        assert np.array_equal(np.asarray(getattr(ms, f)).view(np.uint8), ref[f].view(np.uint8)), f
