"""Density preselection: "preselection-batch-float" / "preselection-batch-int"
(src/Mm/BatchFeatureScorer.cc:238-289, 478-533; src/Mm/DensityClustering.{hh,cc,tcc}).

Tolerances (written here):
  * clustering (cluster of every density, cluster means) and the per-frame cluster selection:
    BIT-EXACT against oracle/presel_oracle.cc, which runs the reference algorithm with libc's
    srand/rand and libstdc++'s std::sort (the tie order of equal distances is std::sort's);
  * preselection-batch-int scores: BIT-EXACT; preselection-batch-float scores: |gpu - ref| <=
    1e-4 * max(1, |ref|) like batch-float (split-f16 kernel), the backoff score exactly.
Parity status: unpinned (gmm_oracle.h); the reference holds no fixtures for these scorers.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import oracle
import rasr_amd as ra

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REL_TOL = 1e-4


# ---------------------------------------------------------------------------
# CPU: host logic and the oracle
# ---------------------------------------------------------------------------
def test_refsort_replay_matches_std_sort(built):
    # the GPU replay of std::sort (rasr_amd/csrc/gmm_refsort.hh) gives std::sort's permutation on
    # tie-heavy inputs, and its heapsort fallback std::partial_sort's
    exe = os.path.join(ROOT, "build", "tests", "refsort_test")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout


@pytest.mark.parametrize("entries,clusters", [(1000, 256), (256, 256), (300, 200), (10, 3), (800000, 256)])
def test_clustering_seeds_are_libc_rand(built, entries, clusters):
    # initializeClusters: srand(1); rand() % nDensities without repetition (DensityClustering.tcc:60-74)
    lib = ra.load_library()
    out = (ctypes.c_uint32 * clusters)()
    assert lib.gmm_density_clustering_seeds(entries, clusters, out) == 0
    r = oracle.libc_rand_sequence(1, 8 * clusters + 64).astype(np.int64)
    ref, used, i = [], set(), 0
    while len(ref) < clusters:
        d = int(r[i]) % entries
        i += 1
        if d not in used:
            used.add(d)
            ref.append(d)
    assert list(out) == ref


def test_clustering_seeds_errors(built):
    lib = ra.load_library()
    out = (ctypes.c_uint32 * 4)()
    assert lib.gmm_density_clustering_seeds(3, 4, out) == -1
    assert lib.gmm_density_clustering_seeds(3, 0, out) == -1


def test_default_preselection_config(built):
    cfg = ra.default_config()  # DensityClustering.cc:19-32
    assert (cfg.clusters, cfg.select_clusters, cfg.clustering_iterations) == (256, 32, 5)
    assert cfg.backoff_score == 40000.0


@pytest.mark.parametrize("kind", ["float", "int"])
def test_oracle_preselection_properties(built, kind):
    ms = ra.synthetic_mixture_set(60, 12, 20, seed=5)
    frames = ra.synthetic_frames(40, 20, seed=6)
    full = (oracle.batch_float_score if kind == "float" else oracle.batch_int_score)(ms, frames)
    o = oracle.OraclePresel(ms, kind, clusters=32, select=32)  # every cluster selected = the batch scorer
    assert np.array_equal(o.score(frames), full)
    o = oracle.OraclePresel(ms, kind, clusters=32, select=4)
    sel = o.select(frames)
    assert (sel.sum(1) == 4).all()
    sc = o.score(frames)
    if kind == "float":
        none = sc == np.float32(40000.0)
        assert none.any()  # mixtures with no selected density: backoff (BatchFeatureScorer.cc:282-288)
        assert (sc[~none] >= full[~none]).all()
    else:
        assert (sc >= full).all()


# ---------------------------------------------------------------------------
# GPU: the product through the C-ABI
# ---------------------------------------------------------------------------
CASES = [
    # (mixtures, densities per mixture, dim, frames, clusters, select)
    (120, 12, 39, 700, 256, 32),
    (50, "ragged", 33, 333, 64, 6),
    (30, 5, 16, 130, 256, 32),      # 150 entries: clusters reduced to 150
    (80, 16, 45, 257, 128, 128),    # everything selected
    (40, 8, 60, 200, 64, 8),        # float: 6 K steps, the 64-frame-wave kernel (128 frames per wave up to 5)
]


def _model(m, k, d, seed=21):
    if k == "ragged":
        k = ra.ragged_counts(m, m * 12, low=1, high=30, seed=seed)
    return ra.synthetic_mixture_set(m, k, d, seed=seed, weights="random")


def _scorer(ms, type_name, n, clusters, select, **kw):
    return ra.Scorer(ms, type_name, max_frames=n, clusters=clusters, select_clusters=select, **kw)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["float", "int"])
@pytest.mark.parametrize("case", CASES)
def test_preselection_parity(gpu, kind, case):
    m, k, d, f, clusters, select = case
    ms = _model(m, k, d)
    frames = ra.synthetic_frames(f, d, seed=31)
    ref = oracle.OraclePresel(ms, kind, clusters=clusters, select=select)
    sc = _scorer(ms, f"preselection-batch-{kind}", f, clusters, select)
    # clustering: bit-exact
    coe, means = sc.density_clustering()
    assert means.shape == ref.cluster_means.shape
    assert np.array_equal(coe, ref.cluster_of_entry)
    assert np.array_equal(means.view(np.uint8), ref.cluster_means.view(np.uint8))
    s, _ = sc.score_host(frames)
    # selection: bit-exact (ties resolved as std::sort does)
    sel = sc.cluster_selection(f)
    ref_sel = ref.select(frames)
    assert np.array_equal(sel, ref_sel), f"{(sel != ref_sel).any(1).sum()} frames select differently"
    ref_s = ref.score(frames, n_threads=8, selection=ref_sel)
    if kind == "int":
        assert np.array_equal(s.view(np.uint32), ref_s.view(np.uint32))
    else:
        backoff = ref_s == np.float32(40000.0)
        assert np.array_equal(s == np.float32(40000.0), backoff)
        err = np.abs(s.astype(np.float64) - ref_s) / np.maximum(1.0, np.abs(ref_s.astype(np.float64)))
        assert err.max() <= REL_TOL, f"max rel err {err.max()}"


@pytest.mark.gpu
def test_preselection_int_ties_across_the_boundary(gpu):
    # u8 features against u8 cluster means: integer distances tie often; the frames whose tied clusters
    # straddle the select-clusters boundary take the std::sort replay on the GPU
    ms = _model(200, 8, 12, seed=4)
    frames = ra.synthetic_frames(512, 12, seed=9)
    ref = oracle.OraclePresel(ms, "int", clusters=256, select=40)
    feats = ref.features(frames).astype(np.int64)
    cm = ref.cluster_means.astype(np.int64)
    dist = ((feats[:, None, :] - cm[None, :, :]) ** 2).sum(-1)
    srt = np.sort(dist, axis=1)
    straddle = (srt[:, 39] == srt[:, 40]).sum()
    assert straddle > 10, "the case must exercise ties at the selection boundary"
    sc = _scorer(ms, "preselection-batch-int", 512, 256, 40)
    s, _ = sc.score_host(frames)
    assert np.array_equal(sc.cluster_selection(512), ref.select(frames))
    assert np.array_equal(s.view(np.uint32), ref.score(frames, n_threads=8).view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["float", "int"])
def test_preselection_score_scale_and_shards(gpu, kind):
    # score_scale multiplies every score (backoff included); a mixture shard is scored with the
    # clustering of the whole mixture set and equals the rows of the full table
    ms = _model(90, 10, 24, seed=8)
    frames = ra.synthetic_frames(200, 24, seed=10)
    full = _scorer(ms, f"preselection-batch-{kind}", 200, 64, 3)
    s_full, _ = full.score_host(frames)
    scaled = _scorer(ms, f"preselection-batch-{kind}", 200, 64, 3, score_scale=0.5)
    s_scaled, _ = scaled.score_host(frames)
    np.testing.assert_array_equal(s_scaled, (np.float32(0.5) * s_full).astype(np.float32))
    part = _scorer(ms, f"preselection-batch-{kind}", 200, 64, 3, mixture_range=(30, 70))
    s_part, _ = part.score_host(frames)
    if kind == "int":
        np.testing.assert_array_equal(s_part, s_full[30:70])
    else:  # the shard's own row-constant offset: equal within the float tolerance
        assert np.array_equal(s_part == np.float32(40000.0), s_full[30:70] == np.float32(40000.0))
        np.testing.assert_allclose(s_part, s_full[30:70], rtol=REL_TOL, atol=REL_TOL)


@pytest.mark.gpu
def test_preselection_errors(gpu):
    ms = _model(10, 4, 16)
    with pytest.raises(RuntimeError):
        _scorer(ms, "preselection-batch-int", 16, 8, 9)  # select-clusters > clusters
    with pytest.raises(RuntimeError):
        _scorer(ms, "preselection-batch-float", 16, 300, 8)  # clusters > 256
    with pytest.raises(RuntimeError):
        ra.Scorer(ms, "preselection-batch-float", max_frames=16, native_f32=True)
    sc = ra.Scorer(ms, "batch-diagonal-maximum-float", max_frames=16)
    with pytest.raises(RuntimeError):
        sc.density_clustering()
