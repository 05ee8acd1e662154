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
