"""gmm_score_host on large batches: the chunked pipeline (frame chunks scored on one stream, the score
table copied out on another), into pageable buffers through the pinned staging ring and into pinned
buffers by direct DMA.  Every path must give the same bits as gmm_score_device on the same frames
(results are per frame, chunking does not change them); the device path itself is checked against the
oracle in test_gpu_parity.py."""
import numpy as np
import pytest
import torch

import rasr_amd as ra


def _device_reference(sc, frames, want_best):
    dev = torch.device("cuda", 0)
    f = len(frames)
    m = sc.n_mixtures()
    x = torch.from_numpy(frames).to(dev)
    s = torch.empty((m, f), dtype=torch.float32, device=dev)
    b = torch.empty((m, f), dtype=torch.int32, device=dev) if want_best else None
    sc.score_device(x, s, b)
    torch.cuda.synchronize()
    return s.cpu().numpy(), (b.cpu().numpy().view(np.uint32) if want_best else None)


# 600 mixtures x 5000 frames x 4 B = 12 MB per table: above the 8 MB pipeline threshold, several
# staging pieces, and (5000 frames) not a multiple of any kernel's frame block
CASES = [("diagonal-maximum", 5000), ("SIMD-diagonal-maximum", 5000), ("batch-diagonal-maximum-int", 17000),
         ("diagonal-maximum", 17000)]


@pytest.fixture(scope="module")
def model():
    return ra.synthetic_mixture_set(600, 8, 33, seed=31)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,nframes", CASES)
def test_pipelined_host_matches_device(gpu, model, kind, nframes):
    frames = ra.synthetic_frames(nframes, 33, seed=nframes)
    sc = ra.Scorer(model, kind, max_frames=nframes)
    want_best = kind != "batch-diagonal-maximum-int"
    ref_s, ref_b = _device_reference(sc, frames, want_best)
    s, b = sc.score_host(frames, want_best=want_best)  # pageable: staging ring
    assert np.array_equal(s.view(np.uint32), ref_s.view(np.uint32))
    if want_best:
        assert np.array_equal(b, ref_b)
    ps = ra.pinned_empty(s.shape, np.float32)
    pb = ra.pinned_empty(s.shape, np.uint32) if want_best else None
    s2, b2 = sc.score_host(frames, want_best=want_best, out=ps, best_out=pb)  # pinned: direct DMA
    assert s2 is ps and np.array_equal(ps.view(np.uint32), ref_s.view(np.uint32))
    if want_best:
        assert np.array_equal(pb, ref_b)


@pytest.mark.gpu
@pytest.mark.parametrize("pinned", [False, True])
def test_pipelined_host_strided_output(gpu, model, pinned):
    """score_stride > n_frames: the columns past n_frames are left untouched."""
    nframes, stride = 9000, 9100
    frames = ra.synthetic_frames(nframes, 33, seed=5)
    sc = ra.Scorer(model, "diagonal-maximum", max_frames=nframes)
    ref_s, ref_b = _device_reference(sc, frames, True)
    m = sc.n_mixtures()
    out = ra.pinned_empty((m, stride), np.float32) if pinned else np.empty((m, stride), np.float32)
    bo = ra.pinned_empty((m, stride), np.uint32) if pinned else np.empty((m, stride), np.uint32)
    out[:] = -7.0
    bo[:] = 123456
    sc.score_host(frames, out=out, best_out=bo)
    assert np.array_equal(out[:, :nframes].view(np.uint32), ref_s.view(np.uint32))
    assert np.array_equal(bo[:, :nframes], ref_b)
    assert (out[:, nframes:] == -7.0).all() and (bo[:, nframes:] == 123456).all()


@pytest.mark.gpu
def test_pipelined_host_preselection(gpu, model):
    """preselection scorers take the pipeline in one chunk (the selection API reports the whole batch)."""
    nframes = 6000
    frames = ra.synthetic_frames(nframes, 33, seed=8)
    sc = ra.Scorer(model, "preselection-batch-int", max_frames=nframes, clusters=32, select_clusters=8)
    ref_s, _ = _device_reference(sc, frames, False)
    sel_dev = sc.cluster_selection(nframes)
    s, _ = sc.score_host(frames, want_best=False)
    assert np.array_equal(s.view(np.uint32), ref_s.view(np.uint32))
    assert np.array_equal(sc.cluster_selection(nframes), sel_dev)


def test_score_host_rejects_bad_outputs(built):
    """argument checks happen before any device work (no GPU needed)."""
    ms = ra.synthetic_mixture_set(4, 2, 5, seed=1)
    sc = object.__new__(ra.Scorer)  # no device handle: the checks must fire first
    sc._lib = ra.load_library()
    sc._h = None
    sc.n_mixtures = lambda: ms.n_mixtures
    frames = ra.synthetic_frames(3, 5, seed=1)
    with pytest.raises(ValueError):
        sc.score_host(frames, out=np.empty((ms.n_mixtures, 2), np.float32))
    with pytest.raises(ValueError):
        sc.score_host(frames, out=np.empty((ms.n_mixtures, 3), np.float64))
    with pytest.raises(ValueError):
        sc.score_host(frames, out=np.empty((ms.n_mixtures, 3), np.float32), best_out=np.empty((1, 3), np.uint32))


def test_pinned_empty_roundtrip(built):
    """gmm_host_alloc needs the HIP runtime but no device work; skip where no device is present."""
    try:
        a = ra.pinned_empty((3, 5), np.uint32)
    except ra.GmmError as e:
        pytest.skip(f"no HIP device for page-locked memory: {e}")
    a[:] = np.arange(15, dtype=np.uint32).reshape(3, 5)
    assert a.sum() == 105 and a.dtype == np.uint32 and a.shape == (3, 5)
    del a


# ------------------------------------------------------------------------------------------------------------
# gmm_score_host_ring / gmm_fetch_best_density: the BatchFeatureScorerBase ring in one call (wrapped or not),
# best densities kept on the device until fetched


def _ring_case(sc, ring, first, n, pinned, keep_best, frame_major=False):
    """keep_best: False (best densities copied with the scores), True (GMM_HOST_KEEP_BEST: computed, fetched
    later) or "lazy" (GMM_HOST_LAZY_BEST: scores only, computed when fetched -- its scores are those of a
    device call without best densities)."""
    m = sc.n_mixtures()
    R = ring.shape[0]
    mk = (lambda shape, dt: ra.pinned_empty(shape, dt)) if pinned else (lambda shape, dt: np.empty(shape, dt))
    shape = (R + 2, m + 3) if frame_major else (m, R + 3)
    out, best = mk(shape, np.float32), mk(shape, np.uint32)
    out[:] = -7.0
    best[:] = 123456
    order = [(first + i) % R for i in range(n)]
    ref_s, ref_b = _device_reference(sc, np.ascontiguousarray(ring[order]), True)
    lazy = keep_best == "lazy"
    if lazy:
        ref_s, _ = _device_reference(sc, np.ascontiguousarray(ring[order]), False)
    cid = sc.score_host_ring(ring, first, n, out, None if keep_best else best, keep_best=keep_best is True,
                             frame_major=frame_major, lazy_best=lazy)
    if keep_best:
        assert (best == 123456).all()  # nothing copied yet
        sc.fetch_best(cid, best)
    pos = np.array(order, dtype=np.int64)
    if frame_major:  # rows = ring positions, columns [0, m) = mixtures
        got_s, got_b = out[pos, :m].T, best[pos, :m].T
        rest = np.ones(shape, bool)
        rest[pos, :m] = False
    else:
        got_s, got_b = out[:, pos], best[:, pos]
        rest = np.ones(shape, bool)
        rest[:, pos] = False
    assert np.array_equal(np.ascontiguousarray(got_s).view(np.uint32), ref_s.view(np.uint32))
    assert np.array_equal(got_b, ref_b)
    assert (out[rest] == -7.0).all() and (best[rest] == 123456).all()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["SIMD-diagonal-maximum", "diagonal-maximum"])
@pytest.mark.parametrize("R,first,n", [(7, 5, 6), (7, 0, 7), (64, 63, 2), (64, 10, 30), (9000, 8000, 9000),
                                       (20000, 3, 17000)])
@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("keep_best", [False, True, "lazy"])
@pytest.mark.parametrize("frame_major", [False, True])
def test_ring_matches_device(gpu, model, kind, R, first, n, pinned, keep_best, frame_major):
    """Small (one chunk) and pipelined (several chunks, the wrap inside a chunk) ring calls, pageable and pinned
    tables, mixture- and frame-major: the ring positions equal gmm_score_device on the frames in ring order;
    everything else is untouched."""
    ring = ra.synthetic_frames(R, 33, seed=R + first)
    sc = ra.Scorer(model, kind, max_frames=max(n, 64))
    _ring_case(sc, ring, first, n, pinned, keep_best, frame_major)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["SIMD-diagonal-maximum", "diagonal-maximum", "diagonal-sum"])
@pytest.mark.parametrize("R,first,n", [(1, 0, 1), (7, 5, 6), (64, 63, 2), (64, 10, 30), (96, 40, 64)])
@pytest.mark.parametrize("keep_best", [False, True, "lazy"])
@pytest.mark.parametrize("frame_major", [False, True])
def test_small_call_page_locked_ring(gpu, model, kind, R, first, n, keep_best, frame_major):
    """Calls of up to 64 frames with a page-locked ring and page-locked tables take the one-stream path
    (scoreHostSmall: the gather kernel reads the ring, the transpose / strided copy kernels write the caller's
    rows over PCIe): bit-identical to gmm_score_device in ring order, wrapped or not, everything else untouched."""
    ring = ra.pinned_empty((R, 33), np.float32)
    ring[:] = ra.synthetic_frames(R, 33, seed=R + first + 1)
    sc = ra.Scorer(model, kind, max_frames=64)
    _ring_case(sc, ring, first, n, True, keep_best, frame_major)


@pytest.mark.gpu
def test_small_call_async_page_locked(gpu, model):
    """GMM_HOST_ASYNC on the small-call path: the call's event is on the one stream; a later call and
    gmm_host_call_wait both see the tables complete."""
    R = 16
    ring = ra.pinned_empty((R, 33), np.float32)
    ring[:] = ra.synthetic_frames(R, 33, seed=5)
    sc = ra.Scorer(model, "diagonal-maximum", max_frames=64)
    m = sc.n_mixtures()
    sync = np.zeros((R, m), np.float32)
    sc.score_host_ring(ring, 0, R, sync, frame_major=True)
    outs = [ra.pinned_empty((R, m), np.float32) for _ in range(3)]
    ids = []
    for i, o in enumerate(outs):  # back to back: each call waits for the previous one by itself
        o[:] = -1.0
        ids.append(sc.score_host_ring(ring, 4 * i, 4, o, frame_major=True, asynchronous=True))
    sc.wait(ids[-1])
    for i, o in enumerate(outs):
        pos = np.arange(4 * i, 4 * i + 4)
        assert np.array_equal(o[pos].view(np.uint32), sync[pos].view(np.uint32))
        rest = np.ones(R, bool)
        rest[pos] = False
        assert (o[rest] == -1.0).all()


@pytest.mark.gpu
def test_fetch_best_after_later_call_is_refused(gpu, model):
    ring = ra.synthetic_frames(16, 33, seed=3)
    sc = ra.Scorer(model, "SIMD-diagonal-maximum", max_frames=16)
    m = sc.n_mixtures()
    out, best = np.empty((m, 16), np.float32), np.empty((m, 16), np.uint32)
    c1 = sc.score_host_ring(ring, 0, 8, out, keep_best=True)
    c2 = sc.score_host_ring(ring, 8, 8, out, keep_best=True)
    assert c2 > c1
    with pytest.raises(ra.GmmError):
        sc.fetch_best(c1, best)  # replaced on the device by c2
    sc.fetch_best(c2, best)
    with pytest.raises(ra.GmmError):  # keep_best with a best table, and a ring shorter than the run
        sc.score_host_ring(ring, 0, 8, out, best, keep_best=True)
    with pytest.raises(ra.GmmError):
        sc.score_host_ring(ring[:4], 0, 8, out)
    # batch types have no assignment: keep_best keeps nothing, fetching is refused
    sb = ra.Scorer(model, "batch-diagonal-maximum-int", max_frames=16)
    cid = sb.score_host_ring(ring, 3, 16, out, keep_best=True)
    with pytest.raises(ra.GmmError):
        sb.fetch_best(cid, best)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["SIMD-diagonal-maximum", "diagonal-maximum", "batch-diagonal-maximum-int"])
def test_async_host_call(gpu, model, kind):
    """GMM_HOST_ASYNC: the call returns once enqueued; after gmm_host_call_wait the pinned tables hold what a
    synchronous call writes.  A later call waits for it by itself; pageable tables are refused."""
    R, first, n = 600, 450, 500  # wraps, several pipeline chunks
    ring = ra.synthetic_frames(R, 33, seed=71)
    sc = ra.Scorer(model, kind, max_frames=n)
    m = sc.n_mixtures()
    sync = np.zeros((R, m), np.float32)
    sc.score_host_ring(ring, first, n, sync, frame_major=True, lazy_best=True)
    out = ra.pinned_empty((R, m), np.float32)
    out[:] = -1.0
    cid = sc.score_host_ring(ring, first, n, out, frame_major=True, lazy_best=True, asynchronous=True)
    sc.wait(cid)
    pos = (first + np.arange(n)) % R
    assert np.array_equal(out[pos].view(np.uint32), sync[pos].view(np.uint32))
    rest = np.ones(R, bool)
    rest[pos] = False
    assert (out[rest] == -1.0).all()
    if kind != "batch-diagonal-maximum-int":  # best densities of the asynchronous call, computed on demand
        best = ra.pinned_empty((R, m), np.uint32)
        sc.fetch_best(cid, best)
        eager = np.zeros((R, m), np.uint32)
        sc.score_host_ring(ring, first, n, np.zeros((R, m), np.float32), eager, frame_major=True)
        assert np.array_equal(best[pos], eager[pos])
    # two asynchronous calls back to back, the second waits for the first; a synchronous one after both
    out2 = ra.pinned_empty((R, m), np.float32)
    c1 = sc.score_host_ring(ring, 0, 100, out, frame_major=True, asynchronous=True)
    c2 = sc.score_host_ring(ring, 100, 100, out2, frame_major=True, asynchronous=True)
    sc.wait(c1)
    sc.wait(c2)
    assert np.array_equal(out2[100:200].view(np.uint32), sync[100:200].view(np.uint32))
    assert np.array_equal(out[0:100].view(np.uint32), sync[0:100].view(np.uint32))
    with pytest.raises(ra.GmmError):
        sc.score_host_ring(ring, 0, 10, np.zeros((R, m), np.float32), frame_major=True, asynchronous=True)
