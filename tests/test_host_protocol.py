"""The C++ host-side scorer classes (rasr_amd/csrc/host/GpuFeatureScorer.hh) driven through the
reference recognizer's protocol (tests/cpp/feature_scorer_driver.cc mirrors
src/Speech/Recognizer.cc:198-206,272-282) against the oracle, frame by frame."""
import os
import subprocess

import numpy as np
import pytest

import oracle
import rasr_amd as ra

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "build", "tests", "feature_scorer_driver")


def _write_model(path, ms):
    with open(path, "wb") as f:
        np.array([ms.dimension, ms.means.shape[0], ms.n_covariances, ms.n_densities, ms.n_mixtures, ms.n_entries],
                 dtype=np.uint32).tofile(f)
        ms.means.astype(np.float32).tofile(f)
        ms.variances.astype(np.float32).tofile(f)
        ms.density_mean.astype(np.uint32).tofile(f)
        ms.density_covariance.astype(np.uint32).tofile(f)
        ms.mixture_offsets.astype(np.uint32).tofile(f)
        ms.mixture_densities.astype(np.uint32).tofile(f)
        ms.mixture_log_weights.astype(np.float64).tofile(f)


def _run(tmp_path, ms, frames, kind, buffer_size, segments, model_file=None, protocol="recognizer", shard_devices=None,
         cache_archive=None, stderr_out=None):
    mp, fp, op = tmp_path / "m.drvmodel", tmp_path / "f.bin", tmp_path / "o.bin"
    if model_file is None:
        _write_model(mp, ms)
    else:
        mp = model_file
    with open(fp, "wb") as f:
        np.array(frames.shape, dtype=np.uint32).tofile(f)
        frames.astype(np.float32).tofile(f)
    env = dict(os.environ)
    if shard_devices:
        env["RASR_DRIVER_SHARD_DEVICES"] = ",".join(str(d) for d in shard_devices)
    if cache_archive:
        env["RASR_DRIVER_CACHE_ARCHIVE"] = str(cache_archive)
    r = subprocess.run([DRIVER, str(mp), str(fp), str(op), kind, str(buffer_size), str(segments), protocol], check=True,
                       timeout=300, env=env, stderr=subprocess.PIPE, text=True)
    if stderr_out is not None:
        stderr_out.append(r.stderr)
    raw = np.fromfile(op, dtype=np.uint32)
    F, M, launches = raw[:3]
    s = raw[3:3 + F * M].view(np.float32).reshape(F, M)
    b = raw[3 + F * M:3 + 2 * F * M].reshape(F, M)
    return s, b, int(launches)


def test_driver_built(built):
    assert os.access(DRIVER, os.X_OK)


@pytest.mark.gpu
@pytest.mark.parametrize("buffer_size", [1, 4, 7])
def test_simd_protocol_bit_exact(gpu, tmp_path, buffer_size):
    ms = ra.synthetic_mixture_set(30, 9, 39, seed=41, weights="random")
    frames = ra.synthetic_frames(53, 39, seed=42)
    s, b, launches = _run(tmp_path, ms, frames, "SIMD-diagonal-maximum", buffer_size, 3)
    ref_s, ref_b, _ = oracle.OracleSimd(ms).score(frames)
    assert np.array_equal(s.T.view(np.uint32), ref_s.view(np.uint32))
    assert np.array_equal(b.T, ref_b)
    if buffer_size > 1:
        assert launches <= 53  # a launch serves every buffered frame


@pytest.mark.gpu
@pytest.mark.parametrize("buffer_size", [1, 64])
@pytest.mark.parametrize("kind", ["SIMD-diagonal-maximum", "batch-diagonal-maximum-int"])
def test_density_sharded_protocol_bit_exact(gpu, tmp_path, kind, buffer_size):
    """The C++ host classes with Configuration::shardDevices (the adapter's "density-shard-devices") = three parts
    on device 0 (copy exchange): the recognizer protocol bit-exact against the oracle, split mixtures included."""
    counts = ra.ragged_counts(30, 30 * 9, low=1, high=20, seed=5)
    ms = ra.synthetic_mixture_set(30, counts, 39, seed=41, weights="random")
    frames = ra.synthetic_frames(53, 39, seed=42)
    s, b, _ = _run(tmp_path, ms, frames, kind, buffer_size, 3, shard_devices=[0, 0, 0])
    if kind == "SIMD-diagonal-maximum":
        ref_s, ref_b, _ = oracle.OracleSimd(ms).score(frames)
        assert np.array_equal(b.T, ref_b)
    else:
        ref_s = oracle.batch_int_score(ms, frames)
    assert np.array_equal(s.T.view(np.uint32), ref_s.view(np.uint32))


@pytest.mark.gpu
def test_batch_int_protocol_bit_exact(gpu, tmp_path):
    ms = ra.synthetic_mixture_set(25, 12, 39, seed=43)
    frames = ra.synthetic_frames(40, 39, seed=44)
    s, _, launches = _run(tmp_path, ms, frames, "batch-diagonal-maximum-int", 4, 2)
    ref = oracle.batch_int_score(ms, frames)
    assert np.array_equal(s.T.view(np.uint32), ref.view(np.uint32))
    assert launches < 40


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["diagonal-maximum", "batch-diagonal-maximum-float"])
def test_float_protocol(gpu, tmp_path, kind):
    ms = ra.synthetic_mixture_set(25, 12, 45, seed=45, weights="random")
    frames = ra.synthetic_frames(31, 45, seed=46)
    s, _, _ = _run(tmp_path, ms, frames, kind, 4, 2)
    ref = oracle.OracleFloat(ms).score(frames)[0] if kind == "diagonal-maximum" else oracle.batch_float_score(ms, frames)
    err = np.abs(s.T.astype(np.float64) - ref) / np.maximum(1, np.abs(ref))
    assert err.max() <= 1e-4


def test_driver_reads_pms_model(built, tmp_path):
    """The driver's model path through MixtureSet::read: a broken .pms file is refused (exit 3)."""
    bad = tmp_path / "bad.pms"
    bad.write_text("#Version: 3.0\n#CovarianceType: DiagonalCovariance\n1 0 0 0 0\n")
    fp = tmp_path / "f.bin"
    with open(fp, "wb") as f:
        np.array([1, 1], dtype=np.uint32).tofile(f)
        np.zeros(1, np.float32).tofile(f)
    r = subprocess.run([DRIVER, str(bad), str(fp), str(tmp_path / "o.bin"), "SIMD-diagonal-maximum", "1", "1"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 3 and "not supported" in r.stderr


@pytest.mark.gpu
def test_simd_protocol_model_from_pms_file(gpu, tmp_path):
    """OfflineRecognizer protocol with the model loaded from a .pms.gz file by the C++ host side."""
    src = ra.synthetic_mixture_set(20, 7, 39, seed=47, weights="random", n_covariances=3)
    path = tmp_path / "model.pms.gz"
    ra.write_mixture_set(str(path), src, 6)
    ms = ra.read_mixture_set(str(path))  # the model as the file holds it
    frames = ra.synthetic_frames(33, 39, seed=48)
    s, b, _ = _run(tmp_path, ms, frames, "SIMD-diagonal-maximum", 5, 2, model_file=path)
    ref_s, ref_b, _ = oracle.OracleSimd(ms).score(frames)
    assert np.array_equal(s.T.view(np.uint32), ref_s.view(np.uint32))
    assert np.array_equal(b.T, ref_b)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["preselection-batch-int", "preselection-batch-float"])
def test_preselection_protocol(gpu, tmp_path, kind):
    # the ring-buffer protocol with the default density-clustering parameters (256 clusters, 32 selected)
    ms = ra.synthetic_mixture_set(40, 12, 39, seed=47, weights="random")
    frames = ra.synthetic_frames(37, 39, seed=48)
    s, _, _ = _run(tmp_path, ms, frames, kind, 4, 2)
    ref = oracle.OraclePresel(ms, "int" if kind.endswith("int") else "float").score(frames)
    if kind.endswith("int"):
        assert np.array_equal(s.T.view(np.uint32), ref.view(np.uint32))
    else:
        err = np.abs(s.T.astype(np.float64) - ref) / np.maximum(1, np.abs(ref))
        assert err.max() <= 1e-4


@pytest.mark.gpu
def test_preselection_cache_archive_protocol(gpu, tmp_path):
    # Gpu::Configuration::cacheArchive (the adapter's "density-clustering.cache-archive"): the first drop-in scorer
    # builds and writes the clustering, the second reads it -- same scores, bit-exact against the oracle
    ms = ra.synthetic_mixture_set(40, 12, 39, seed=47, weights="random")
    frames = ra.synthetic_frames(37, 39, seed=48)
    archive = tmp_path / "global.cache"
    err = []
    s1, _, _ = _run(tmp_path, ms, frames, "preselection-batch-int", 4, 2, cache_archive=archive, stderr_out=err)
    s2, _, _ = _run(tmp_path, ms, frames, "preselection-batch-int", 4, 2, cache_archive=archive, stderr_out=err)
    assert "clustering: written" in err[0] and "clustering: cached" in err[1], err
    assert archive.exists()
    ref = oracle.OraclePresel(ms, "int").score(frames)
    assert np.array_equal(s1.T.view(np.uint32), ref.view(np.uint32))
    assert np.array_equal(s2.view(np.uint32), s1.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("kind,buffer_size", [("SIMD-diagonal-maximum", 1), ("SIMD-diagonal-maximum", 6),
                                              ("batch-diagonal-maximum-int", 4), ("diagonal-maximum", 5)])
def test_feature_scorer_node_dump(gpu, tmp_path, kind, buffer_size):
    """Speech::FeatureScorerNode (src/Speech/FeatureScorerNode.cc:95-162), the reference's score dump: every
    frame yields -score(e) for all nEmissions() mixtures, in frame order, with finalize() + reset() after each
    segment.  Compared with the oracle's scores negated."""
    ms = ra.synthetic_mixture_set(28, 10, 39, seed=49, weights="random")
    frames = ra.synthetic_frames(47, 39, seed=50)
    s, b, _ = _run(tmp_path, ms, frames, kind, buffer_size, 3, protocol="node")
    if kind == "SIMD-diagonal-maximum":
        ref_s, ref_b, _ = oracle.OracleSimd(ms).score(frames)
        assert np.array_equal(s.T.view(np.uint32), (-ref_s).view(np.uint32))
        assert np.array_equal(b.T, ref_b)
    elif kind == "batch-diagonal-maximum-int":
        assert np.array_equal(s.T.view(np.uint32), (-oracle.batch_int_score(ms, frames)).view(np.uint32))
    else:
        ref = -oracle.OracleFloat(ms).score(frames)[0]
        assert (np.abs(s.T.astype(np.float64) - ref) / np.maximum(1, np.abs(ref))).max() <= 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["SIMD-diagonal-maximum", "diagonal-maximum"])
def test_protocol_model_from_estimator_file(gpu, tmp_path, kind):
    """A model a trainer wrote as a binary estimator file (the reference's default reader, MixtureSetReader.cc:52-74)
    loads through the C++ host side (Mm::Gpu::MixtureSet::read) and scores through the recognizer protocol."""
    from oracle import estimator as est
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "estimator", "model.mix")
    ms = ra.read_mixture_set(path)  # the estimated model
    frames = ra.synthetic_frames(41, ms.dimension, seed=51) * 2
    s, b, _ = _run(tmp_path, ms, frames, kind, 6, 2, model_file=path)
    if kind == "SIMD-diagonal-maximum":
        ref_s, ref_b, _ = oracle.OracleSimd(ms).score(frames)
        assert np.array_equal(s.T.view(np.uint32), ref_s.view(np.uint32))
        assert np.array_equal(b.T, ref_b)
    else:
        ref = oracle.OracleFloat(ms).score(frames)[0]
        assert (np.abs(s.T.astype(np.float64) - ref) / np.maximum(1, np.abs(ref))).max() <= 1e-4
    del est


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["SIMD-diagonal-maximum", "diagonal-maximum"])
def test_delayed_consumer_unbuffered(gpu, tmp_path, kind):
    """A consumer that reads each context only after 3 more frames were scored (RecognizerDelayHandler,
    src/Speech/DelayedRecognizer.cc:65-135): scores come from the context's own page-locked slot.  The first four
    contexts were scored before any bestDensity() (scores only); their frames were replaced on the device by the
    later ones, so their best densities come from scoring each frame again (4 launches).  From the first
    bestDensity() on every getScorer() computes the best densities in its own launch (launches = F + 4)."""
    ms = ra.synthetic_mixture_set(30, 9, 39, seed=52, weights="random")
    frames = ra.synthetic_frames(29, 39, seed=53)
    s, b, launches = _run(tmp_path, ms, frames, kind, 1, 2, protocol="delayed")
    if kind == "SIMD-diagonal-maximum":
        ref_s, ref_b, _ = oracle.OracleSimd(ms).score(frames)
        assert np.array_equal(s.T.view(np.uint32), ref_s.view(np.uint32))
        assert np.array_equal(b.T, ref_b)
    else:
        ref_s, ref_b = oracle.OracleFloat(ms).score(frames)[:2]
        assert (np.abs(s.T.astype(np.float64) - ref_s) / np.maximum(1, np.abs(ref_s))).max() <= 1e-4
    assert launches == 29 + 4


@pytest.mark.gpu
@pytest.mark.parametrize("kind,buffer_size", [("SIMD-diagonal-maximum", 64), ("SIMD-diagonal-maximum", 100),
                                              ("batch-diagonal-maximum-int", 64), ("diagonal-maximum", 64),
                                              ("batch-diagonal-maximum-float", 80)])
def test_prefetch_search_protocol(gpu, tmp_path, kind, buffer_size):
    """Buffers of 64 frames and more prefetch: the newest half of the ring goes to the GPU as a GMM_HOST_ASYNC
    call (score-only kernels, GMM_HOST_LAZY_BEST) while older positions are consumed.  The recognizer's sequence
    reading score(e) only, over three segments (reset between them): the same scores as the oracle, fewer launches
    than frames."""
    ms = ra.synthetic_mixture_set(40, ra.ragged_counts(40, 40 * 12, low=1, high=30, seed=61), 39, seed=61,
                                  weights="random")
    frames = ra.synthetic_frames(701, 39, seed=62)
    s, b, launches = _run(tmp_path, ms, frames, kind, buffer_size, 3, protocol="search")
    assert (b == 0xFFFFFFFF).all()
    if kind == "SIMD-diagonal-maximum":
        ref = oracle.OracleSimd(ms).score(frames)[0]
    elif kind == "batch-diagonal-maximum-int":
        ref = oracle.batch_int_score(ms, frames)
    elif kind == "diagonal-maximum":
        ref = oracle.OracleFloat(ms).score(frames)[0]
    else:
        ref = oracle.batch_float_score(ms, frames)
    if kind in ("SIMD-diagonal-maximum", "batch-diagonal-maximum-int"):
        assert np.array_equal(s.T.view(np.uint32), ref.view(np.uint32))
    else:
        err = np.abs(s.T.astype(np.float64) - ref) / np.maximum(1, np.abs(ref))
        assert err.max() <= 1e-4
    assert launches < 701 // 8


@pytest.mark.gpu
@pytest.mark.parametrize("protocol", ["recognizer", "node"])
def test_prefetch_then_best_densities(gpu, tmp_path, protocol):
    """A buffer that prefetches, read by a consumer that asks bestDensity(e) too (the aligners; the node's dump):
    from the first bestDensity() on the prefetched calls carry the best densities too; the scores and best densities
    stay bit-exact."""
    ms = ra.synthetic_mixture_set(30, 9, 39, seed=63, weights="random")
    frames = ra.synthetic_frames(260, 39, seed=64)
    s, b, _ = _run(tmp_path, ms, frames, "SIMD-diagonal-maximum", 64, 2, protocol=protocol)
    ref_s, ref_b, _ = oracle.OracleSimd(ms).score(frames)
    sign = -1.0 if protocol == "node" else 1.0
    assert np.array_equal((sign * s.T).astype(np.float32).view(np.uint32), ref_s.view(np.uint32))
    assert np.array_equal(b.T, ref_b)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["SIMD-diagonal-maximum", "diagonal-maximum"])
def test_prefetch_then_late_best_densities(gpu, tmp_path, kind):
    """score(e) only for the first half of the frames (prefetch runs, several asynchronous calls), then
    bestDensity(e) as well: the best densities of positions whose call is no longer the newest come from one
    refill of the buffer, and equal the oracle's (SIMD bit-exact; float: the scores within 1e-4, the best
    densities where the two best candidates are not a near tie)."""
    ms = ra.synthetic_mixture_set(30, 9, 39, seed=65, weights="random")
    F = 400
    frames = ra.synthetic_frames(F, 39, seed=66)
    s, b, _ = _run(tmp_path, ms, frames, kind, 64, 1, protocol="late")
    if kind == "SIMD-diagonal-maximum":
        ref_s, ref_b, _ = oracle.OracleSimd(ms).score(frames)
        assert np.array_equal(s.T.view(np.uint32), ref_s.view(np.uint32))
    else:
        ref_s, ref_b = oracle.OracleFloat(ms).score(frames)
        assert (np.abs(s.T.astype(np.float64) - ref_s) / np.maximum(1, np.abs(ref_s))).max() <= 1e-4
    assert (b[: F // 2] == 0xFFFFFFFF).all()
    agree = (b.T[:, F // 2:] == ref_b[:, F // 2:]).mean()
    assert agree == 1.0 if kind == "SIMD-diagonal-maximum" else agree > 0.99


def _near_tie_ok(ms, frames, b, ref_b, asked):
    """Float types: every asked best density equals the restatement's, or the two densities' scores (f64 here) are
    within the float contract (1e-4 relative) -- a near tie either may name."""
    t, e = np.nonzero(asked & (b != ref_b.T))
    for ti, ei in zip(t, e):
        lo = int(ms.mixture_offsets[ei])
        sc = []
        for d in (int(b[ti, ei]), int(ref_b[ei, ti])):
            dns = ms.mixture_densities[lo + d]
            var = ms.variances[ms.density_covariance[dns]].astype(np.float64)
            dist = (((frames[ti] - ms.means[ms.density_mean[dns]]) / np.sqrt(var)) ** 2).sum()
            sc.append(-2.0 * ms.mixture_log_weights[lo + d] + oracle.gauss_log_norm(var.astype(np.float32)) + dist)
        assert abs(sc[0] - sc[1]) <= 1e-4 * max(1.0, abs(sc[1])), (ti, ei, b[ti, ei], ref_b[ei, ti], sc)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,buffer_size", [("SIMD-diagonal-maximum", 1), ("SIMD-diagonal-maximum", 7),
                                              ("SIMD-diagonal-maximum", 64), ("diagonal-maximum", 1),
                                              ("diagonal-maximum", 64), ("diagonal-sum", 64)])
def test_aligner_sparse_best_densities(gpu, tmp_path, kind, buffer_size):
    """An aligner's read (AbstractMixtureSetEstimator.cc:370-384): score(e) of every emission and
    bestDensity(e) of 1-10 emissions per frame.  The positions of calls made before the first bestDensity() answer
    it one pair at a time (gmm_best_density_pairs, up to kSparseMax pairs per call, then the call's whole table);
    every later call carries the best densities (prefetches included).  SIMD bit-exact against the restatement,
    the float types within the near-tie rule; the frames the consumer never asked stay 0xffffffff."""
    counts = ra.ragged_counts(30, 30 * 9, low=1, high=90, seed=67)  # mixtures of 1 .. 90 densities (two waves' scan)
    ms = ra.synthetic_mixture_set(30, counts, 39, seed=67, weights="random")
    frames = ra.synthetic_frames(300, 39, seed=68)
    s, b, _ = _run(tmp_path, ms, frames, kind, buffer_size, 2, protocol="aligner")
    asked = b != 0xFFFFFFFF
    assert asked.sum() >= 300 and asked.sum(axis=1).max() <= 10
    if kind == "SIMD-diagonal-maximum":
        ref_s, ref_b, _ = oracle.OracleSimd(ms).score(frames)
        assert np.array_equal(s.T.view(np.uint32), ref_s.view(np.uint32))
        assert np.array_equal(b[asked], ref_b.T[asked])
    else:
        of = oracle.OracleFloatSum(ms) if kind == "diagonal-sum" else oracle.OracleFloat(ms)
        ref_s, ref_b = of.score(frames)[:2]
        assert (np.abs(s.T.astype(np.float64) - ref_s) / np.maximum(1, np.abs(ref_s))).max() <= 1e-4
        _near_tie_ok(ms, frames.astype(np.float64), b, ref_b, asked)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,buffer_size", [("diagonal-maximum", 1), ("diagonal-maximum", 8), ("diagonal-sum", 8)])
def test_best_density_memoized_across_table_switch(gpu, tmp_path, kind, buffer_size):
    """bestDensity(e) of one (frame, e) is answered once (the reference's
    CachedAssigningContextScorer memoizes it, AssigningFeatureScorer.hh:110-121).  Mixture 0 holds a planted near tie
    -- two densities with the same mean, the second better by 1e-4 in -2 log c, below the keyed table's resolution
    but above f32's -- so the single-pair answer (the reference's arithmetic: density 1) and the keyed table's
    differ.  The consumer asks bestDensity(0), then every other emission (past kSparseMax single-pair answers: the
    call's whole keyed table is fetched), then bestDensity(0) again: both answers are the same, and the first frame's
    is the reference's."""
    ms = ra.synthetic_mixture_set(40, 4, 39, seed=69, weights="random")
    ms.means[1] = ms.means[0]
    ms.means[2:4] = ms.means[0] + 30.0  # never the best: the tie is between densities 0 and 1 in every frame
    lw = np.log(0.25)
    ms.mixture_log_weights[:4] = [lw, lw + 5e-5, np.log(0.3), np.log(0.2) - 1e-2]
    frames = ra.synthetic_frames(24, 39, seed=70)
    err = []
    s, b, _ = _run(tmp_path, ms, frames, kind, buffer_size, 1, protocol="memo", stderr_out=err)
    assert "memo mismatches: 0" in err[0], err[0]
    of = oracle.OracleFloatSum(ms) if kind == "diagonal-sum" else oracle.OracleFloat(ms)
    ref_b = of.score(frames)[1]
    assert (ref_b[0] == 1).all()  # the planted tie: the reference names density 1
    assert b[0, 0] == 1
    # the keyed table (what the fetched table holds) names density 0 for this tie: the memo is what kept the answer
    sc = ra.Scorer(ms, kind, max_frames=24)
    assert (sc.score_host(frames)[1][0] == 0).any()
    assert (b != 0xFFFFFFFF).all()
