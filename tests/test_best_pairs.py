"""Sparse best densities (gmm_best_density_pairs / gmm_best_density_pairs_device, gmm_kernels_pairs.hip).

An aligner asks bestDensity(e) for a few emissions per frame (AssigningFeatureScorer.hh:110-121,
AbstractMixtureSetEstimator.cc:370-384).  The pairs call answers a list of (frame, mixture) pairs from frames still
on the device, in the reference's own arithmetic and scan order:
* SIMD-diagonal-maximum: bit-exact against the restatement (oracle/gmm_oracle.c orc_simd_score) -- ragged, empty and
  large (> 64 densities: several scan blocks) mixtures, several covariances, exact ties (duplicated densities), shards,
  the quantizer's edge frames;
* diagonal-maximum: the restatement's arithmetic (the direct scorer's reference-order distance, f64 sum, the
  f32-stored best): equal to orc_float_score's best densities;
* diagonal-sum: the f32 density scores of GaussDiagonalSumFeatureScorer (cc:238-261), minimum by a strict compare;
  equal to orc_float_sum_score's best densities except on near ties (1e-4 relative).
Also: ring positions of a host call (wrapped ring), errors (replaced call, position or mixture out of range, batch
types), and the device variant on torch tensors."""
import numpy as np
import pytest

import oracle
import rasr_amd as ra

pytestmark = pytest.mark.gpu


def _counts(m, lo, hi, seed):
    return np.random.default_rng(seed).integers(lo, hi + 1, size=m)


def _all_pairs(nf, nm):
    f, m = np.meshgrid(np.arange(nf, dtype=np.uint32), np.arange(nm, dtype=np.uint32), indexing="ij")
    return f.ravel(), m.ravel()


def _host_pairs(sc, frames, pos, mix, ring=None, first=0):
    """One lazy host call over `frames` (ring rows at first, first + 1, ... mod R), then the pairs."""
    f = frames.shape[0]
    R = f if ring is None else ring
    ringbuf = np.zeros((R, frames.shape[1]), np.float32)
    for i in range(f):
        ringbuf[(first + i) % R] = frames[i]
    out = np.empty((sc.n_mixtures(), R), np.float32)
    cid = sc.score_host_ring(ringbuf, first, f, out, lazy_best=True)
    return sc.best_pairs(cid, pos, mix), out


SIMD_CASES = [
    # mixtures, (low, high) densities per mixture, dim, covariances, frames
    (40, (0, 9), 39, 1, 37),      # empty and tiny mixtures
    (12, (60, 200), 39, 1, 20),   # several 64-entry scan blocks
    (20, (1, 40), 80, 3, 25),     # two K steps of the scorer, several covariances
    (30, (1, 20), 16, 1, 64),
]


@pytest.mark.parametrize("case", SIMD_CASES)
def test_simd_pairs_bit_exact(gpu, case):
    m, (lo, hi), d, c, f = case
    ms = ra.synthetic_mixture_set(m, _counts(m, lo, hi, m + d), d, seed=71 + m, n_covariances=c, weights="random")
    frames = ra.synthetic_frames(f, d, seed=72)
    _, ref_b, _ = oracle.OracleSimd(ms).score(frames)
    sc = ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=f)
    pf, pm = _all_pairs(f, m)
    got, _ = _host_pairs(sc, frames, pf, pm)
    assert np.array_equal(got, ref_b[pm, pf])
    empty = np.diff(ms.mixture_offsets) == 0
    if empty.any():
        assert (got[empty[pm]] == 0xFFFFFFFF).all()


def test_simd_pairs_ties_and_edge_frames(gpu):
    """Duplicated densities (exact ties: the lower index), frames at the quantizer's limits, NaN / inf frames."""
    rng = np.random.default_rng(9)
    base = ra.synthetic_mixture_set(10, 12, 39, seed=73, weights="uniform")
    means = base.means.copy()
    means[3] = means[2]
    means[7] = means[2]
    ms = ra.MixtureSet(means=means, variances=base.variances, density_mean=base.density_mean,
                       density_covariance=base.density_covariance, mixture_offsets=base.mixture_offsets,
                       mixture_densities=base.mixture_densities, mixture_log_weights=base.mixture_log_weights)
    frames = rng.standard_normal((12, 39)).astype(np.float32)
    frames[1] = means[2]
    frames[2] = 1e6
    frames[3] = -1e6
    frames[4, 5] = np.nan
    frames[5, 0] = np.inf
    _, ref_b, _ = oracle.OracleSimd(ms).score(frames)
    sc = ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=12)
    pf, pm = _all_pairs(12, 10)
    got, _ = _host_pairs(sc, frames, pf, pm)
    assert np.array_equal(got, ref_b[pm, pf])


def test_simd_pairs_shard_and_ring(gpu):
    """A mixture shard (mixture_range): mixture indices are the shard's; positions of a wrapped ring."""
    ms = ra.synthetic_mixture_set(50, _counts(50, 1, 30, 3), 39, seed=74, weights="random")
    frames = ra.synthetic_frames(20, 39, seed=75)
    _, ref_b, _ = oracle.OracleSimd(ms).score(frames)
    sc = ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=32, mixture_range=(10, 35))
    R, first = 32, 25  # frames land at ring positions 25 .. 31, 0 .. 12
    pos = (first + np.arange(20, dtype=np.uint32)) % R
    pf, pm = _all_pairs(20, 25)
    got, _ = _host_pairs(sc, frames, pos[pf], pm, ring=R, first=first)
    assert np.array_equal(got, ref_b[10 + pm, pf])


@pytest.mark.parametrize("kind", ["diagonal-maximum", "diagonal-sum"])
@pytest.mark.parametrize("case", [(30, (1, 40), 39, 1, 33), (10, (70, 150), 45, 2, 9), (16, (0, 5), 13, 1, 20)])
def test_float_pairs(gpu, kind, case):
    m, (lo, hi), d, c, f = case
    if kind == "diagonal-sum":
        c = 1  # the diagonal-sum scorer runs on the one-covariance split kernel only
    ms = ra.synthetic_mixture_set(m, _counts(m, lo, hi, m + d), d, seed=76 + m, n_covariances=c, weights="random")
    frames = ra.synthetic_frames(f, d, seed=77)
    of = oracle.OracleFloatSum(ms) if kind == "diagonal-sum" else oracle.OracleFloat(ms)
    ref_b = of.score(frames)[1]
    sc = ra.Scorer(ms, kind, max_frames=f)
    pf, pm = _all_pairs(f, m)
    got, _ = _host_pairs(sc, frames, pf, pm)
    want = ref_b[pm, pf]
    assert np.array_equal(got, want)  # the restatement's own arithmetic and order, both kinds
    # the keyed table scorer agrees wherever its candidates are not a near tie
    _, kb = sc.score_host(frames)
    assert (kb[pm, pf] == got).mean() > 0.99


def test_float_pairs_scales(gpu):
    """mixture-weight-scale and gaussian-scale enter the pairs' scores as the restatement's."""
    ms = ra.synthetic_mixture_set(20, _counts(20, 2, 30, 5), 39, seed=78, weights="random")
    frames = ra.synthetic_frames(15, 39, seed=79)
    ref_b = oracle.OracleFloat(ms, mixture_weight_scale=3.0, gaussian_scale=0.25).score(frames)[1]
    sc = ra.Scorer(ms, "diagonal-maximum", max_frames=15, mixture_weight_scale=3.0, gaussian_scale=0.25)
    pf, pm = _all_pairs(15, 20)
    got, _ = _host_pairs(sc, frames, pf, pm)
    assert np.array_equal(got, ref_b[pm, pf])


def test_pairs_errors(gpu):
    ms = ra.synthetic_mixture_set(8, 5, 39, seed=80)
    frames = ra.synthetic_frames(6, 39, seed=81)
    sc = ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=8)
    ring = np.zeros((8, 39), np.float32)
    ring[:6] = frames
    out = np.empty((8, 8), np.float32)
    cid = sc.score_host_ring(ring, 0, 6, out, lazy_best=True)
    with pytest.raises(RuntimeError, match="position"):
        sc.best_pairs(cid, [6], [0])  # ring position 6 was not scored by the call
    with pytest.raises(RuntimeError, match="mixture"):
        sc.best_pairs(cid, [0], [8])
    assert sc.best_pairs(cid, [], []).size == 0
    cid2 = sc.score_host_ring(ring, 0, 6, out, lazy_best=True)
    with pytest.raises(RuntimeError, match="replaced"):
        sc.best_pairs(cid, [0], [0])
    sc.best_pairs(cid2, [0], [0])
    bi = ra.Scorer(ms, "batch-diagonal-maximum-int", max_frames=8)
    cid3 = bi.score_host_ring(ring, 0, 6, out)
    with pytest.raises(RuntimeError, match="batch types"):
        bi.best_pairs(cid3, [0], [0])


@pytest.mark.parametrize("kind", ["SIMD-diagonal-maximum", "diagonal-maximum"])
def test_pairs_device(gpu, kind):
    """gmm_best_density_pairs_device on torch tensors: strided frames, random pairs, out-of-range pairs -> none."""
    import torch
    ms = ra.synthetic_mixture_set(25, _counts(25, 1, 70, 7), 39, seed=82, weights="random")
    frames = ra.synthetic_frames(40, 39, seed=83)
    ref_b = (oracle.OracleSimd(ms).score(frames)[1] if kind.startswith("SIMD") else oracle.OracleFloat(ms).score(frames)[1])
    sc = ra.Scorer(ms, kind, max_frames=40)
    x = torch.zeros((40, 48), dtype=torch.float32, device=gpu)
    x[:, :39] = torch.from_numpy(frames).to(gpu)
    rng = np.random.default_rng(4)
    pf = rng.integers(0, 40, size=500).astype(np.int32)
    pm = rng.integers(0, 25, size=500).astype(np.int32)
    pf[:3] = [40, 0, 1 << 30]  # out of range: frame, ok, frame
    pm[:3] = [0, 25, 3]        # ok, mixture out of range, ok
    tf, tm = torch.from_numpy(pf).to(gpu), torch.from_numpy(pm).to(gpu)
    out = torch.full((500,), 7, dtype=torch.int32, device=gpu)
    sc.best_pairs_device(x, tf, tm, out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    assert (got[:3] == 0xFFFFFFFF).all()
    assert np.array_equal(got[3:], ref_b[pm[3:], pf[3:]])

