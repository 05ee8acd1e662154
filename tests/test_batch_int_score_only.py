"""batch-diagonal-maximum-int / -fast on the score-only class layout (gmm_prepare.cc buildClassLayout,
gmm_kernels_i8.hip SCORE_ONLY): rows grouped by the parity of their constant Q = c + sum a'^2 over a tile's lane
groups, h = Q >> 1 as the matrix core's accumulator input, one v_min3 per two candidates, 2 min(v) + p per lane
group at the mixture end.  Bit-exact against the oracle (BatchIntFeatureScorer, BatchFeatureScorer.cc:339-470)
and against the (score, density) key layout (GMM_FLAG_FULL_KEYS) on ragged, tiny and empty mixtures, shards,
uneven frame counts; the dimensions above 64 (two K steps) and models outside the layout's range take the key
layout."""
import numpy as np
import pytest

import oracle
import rasr_amd as ra


def _scores(ms, frames, kind="batch-diagonal-maximum-int", **kw):
    sc = ra.Scorer(ms, kind, max_frames=max(len(frames), 1), **kw)
    return sc.score_host(frames, want_best=False)[0]


def _same(a, b):
    d = np.flatnonzero(a.view(np.uint32).ravel() != b.view(np.uint32).ravel())
    assert d.size == 0, f"{d.size} scores differ; first {d[:5]}"


CASES = [
    # mixtures, densities per mixture (int, or (low, high) ragged), dim, weights, frames
    (60, (1, 40), 39, "random", 301),
    (200, (0, 9), 39, "random", 130),      # empty and tiny mixtures
    (40, 160, 39, "uniform", 257),
    (33, (50, 256), 45, "random", 96),
    (64, 16, 16, "random", 513),
    (25, 3, 64, "random", 77),
    (12, 7, 80, "uniform", 200),            # two K steps: key layout
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_score_only_bit_exact(gpu, case):
    m, k, d, w, f = case
    if isinstance(k, tuple) and k[0] == 0:  # empty mixtures included
        k = np.random.default_rng(m).integers(0, k[1] + 1, size=m)
    elif isinstance(k, tuple):
        k = ra.ragged_counts(m, m * (k[0] + k[1]) // 2, low=k[0], high=k[1], seed=m)
    ms = ra.synthetic_mixture_set(m, k, d, seed=17 + m, weights=w)
    frames = ra.synthetic_frames(f, d, seed=18)
    ref = oracle.batch_int_score(ms, frames, n_threads=8)
    s = _scores(ms, frames)
    _same(s, ref)
    _same(_scores(ms, frames, full_keys=True), ref)


@pytest.mark.gpu
def test_score_only_shards_and_scale(gpu):
    ms = ra.synthetic_mixture_set(90, ra.ragged_counts(90, 90 * 30, low=1, high=60, seed=5), 39, seed=6,
                                  weights="random")
    frames = ra.synthetic_frames(200, 39, seed=7)
    ref = oracle.batch_int_score(ms, frames, n_threads=8)
    for lo, hi in ((0, 45), (45, 90), (10, 11)):
        s = _scores(ms, frames, mixture_range=(lo, hi))
        _same(s[: hi - lo], ref[lo:hi])
    s = _scores(ms, frames, score_scale=0.75)
    _same(s, (np.float32(0.75) * ref).astype(np.float32))


@pytest.mark.gpu
@pytest.mark.parametrize("d", [33, 39, 48])
def test_batch_fast_score_only(gpu, d):
    ms = ra.synthetic_mixture_set(50, ra.ragged_counts(50, 50 * 20, low=1, high=40, seed=d), d, seed=d,
                                  weights="random")
    frames = ra.synthetic_frames(150, d, seed=d + 1)
    _same(_scores(ms, frames, "batch-diagonal-maximum-fast"), oracle.batch_fast_score(ms, frames))


@pytest.mark.gpu
def test_score_only_device_strided(gpu):
    import torch
    ms = ra.synthetic_mixture_set(70, ra.ragged_counts(70, 70 * 20, low=1, high=40, seed=9), 39, seed=9,
                                  weights="random")
    frames = ra.synthetic_frames(333, 39, seed=10)
    ref = oracle.batch_int_score(ms, frames, n_threads=8)
    sc = ra.Scorer(ms, "batch-diagonal-maximum-int", max_frames=400)
    fr = torch.zeros((333, 48), dtype=torch.float32, device=gpu)
    fr[:, :39] = torch.from_numpy(frames).to(gpu)
    out = torch.full((70, 350), -1.0, dtype=torch.float32, device=gpu)
    sc.score_device(fr, out)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    _same(np.ascontiguousarray(o[:, :333]), ref)
    assert (o[:, 333:] == -1.0).all()
