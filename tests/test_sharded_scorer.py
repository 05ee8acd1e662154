"""Density-sharded scorer for a C / C++ caller (gmm_scorer_create_sharded, BASELINE config 4 in one process):
part r of the density shard plan on devices[r], mixtures split between parts reduced per frame over packed
keys, the full table assembled on devices[0].

CPU: the C++ shard plan (gmm_density_shard_plan, rasr_amd/csrc/gmm_shard.cc) equals the Python plan
(rasr_amd/parallel.py density_shards) on ragged, empty-mixture and tiny models; argument checks.
GPU: N parts on ONE GPU with the copy exchange (AUTO's choice when all parts share a GPU; the RCCL exchange on one
GPU, a one-rank all-reduce after an on-device fold, is tests/test_rccl_exchange.py) against the
unsharded scorer -- bit for bit for the quantized types (scores and best densities), within the float contract
for diagonal-maximum (checked against the oracle as tests/test_density_sharded.py does) -- through
gmm_score_host, gmm_score_host_ring (frame-major, keep-best + fetch) and gmm_score_device; N = 1 is the
unsharded scorer itself."""
import ctypes

import numpy as np
import pytest

import rasr_amd as ra
from rasr_amd import _capi, parallel


def _c_plan(offsets, world):
    lib = _capi.load_library()
    off = np.ascontiguousarray(offsets, dtype=np.uint32)
    table = np.zeros((world, 5), dtype=np.uint32)
    split = np.zeros(max(world - 1, 1), dtype=np.uint32)
    n = ctypes.c_uint32()
    _capi.check(lib.gmm_density_shard_plan(off.ctypes.data_as(ctypes.c_void_p), len(off) - 1, world,
                                           table.ctypes.data_as(ctypes.c_void_p), split.ctypes.data_as(ctypes.c_void_p),
                                           ctypes.byref(n)), "gmm_density_shard_plan")
    return table, list(split[: n.value])


def _offset_cases():
    rng = np.random.default_rng(11)
    yield np.concatenate([[0], np.cumsum(ra.ragged_counts(60, 60 * 14, low=1, high=40, seed=3))])
    yield np.concatenate([[0], np.cumsum(ra.ragged_counts(5000, 800_000, seed=99))])
    yield np.arange(0, 5001 * 160, 160)  # config 4: boundaries on mixture boundaries
    for _ in range(20):
        counts = rng.integers(0, 6, size=int(rng.integers(1, 30)))  # empty mixtures, tiny sets
        yield np.concatenate([[0], np.cumsum(counts)])
    yield np.array([0, 0, 0])  # no entries at all
    yield np.array([0, 3])     # one mixture


def test_shard_plan_matches_python_plan(built):
    for offsets in _offset_cases():
        for world in (1, 2, 3, 5, 8, 9):
            table, split = _c_plan(offsets, world)
            ref = parallel.density_shards(offsets, world)
            for r, sh in enumerate(ref):
                assert tuple(table[r]) == (*sh["entries"], *sh["mixtures"], sh["first_offset"]), (offsets, world, r)
            assert split == parallel.split_mixtures(ref)
            assert len(split) <= world - 1


def test_shard_plan_rejects_bad_arguments(built):
    lib = _capi.load_library()
    off = np.array([0, 4, 2], dtype=np.uint32)  # decreasing
    n = ctypes.c_uint32()
    assert lib.gmm_density_shard_plan(off.ctypes.data_as(ctypes.c_void_p), 2, 2, None, None, ctypes.byref(n)) == \
        -1  # GMM_ERR_INVALID_ARGUMENT
    assert lib.gmm_density_shard_plan(off.ctypes.data_as(ctypes.c_void_p), 2, 0, None, None, ctypes.byref(n)) == \
        -1  # GMM_ERR_INVALID_ARGUMENT


# ------------------------------------------------------------------------------------------------------- GPU
QUANTIZED = ["SIMD-diagonal-maximum", "batch-diagonal-maximum-int"]
KINDS = QUANTIZED + ["diagonal-maximum", "batch-diagonal-maximum-float"]


def _ragged_model(n_mix=60, total=60 * 14, seed=5):
    counts = ra.ragged_counts(n_mix, total, low=1, high=40, seed=3)
    return ra.synthetic_mixture_set(n_mix, counts, 39, seed=seed, weights="random")


def _compare(kind, ms, frames, s, b, ref_s, ref_b):
    """Quantized: bit for bit against the unsharded scorer.  Float: the oracle with the float contract
    (1e-4 relative; diagonal-maximum's best densities may differ only at near ties), as
    tests/test_density_sharded.py checks the Python layout."""
    if kind in QUANTIZED:
        assert np.array_equal(s.view(np.uint32), ref_s.view(np.uint32))
        if kind == "SIMD-diagonal-maximum":
            assert np.array_equal(b, ref_b)
    elif kind == "diagonal-maximum":
        from test_density_sharded import _check_against_oracle
        _check_against_oracle(ms, kind, frames, s, b)
    else:
        import oracle
        ref = oracle.batch_float_score(ms, frames, n_threads=16)
        err = np.abs(s.astype(np.float64) - ref) / np.maximum(1.0, np.abs(ref.astype(np.float64)))
        assert err.max() <= 1e-4, f"max rel err {err.max()}"


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("kind", KINDS)
def test_sharded_host_equals_unsharded(gpu, kind, world):
    ms = _ragged_model()
    frames = ra.synthetic_frames(300, 39, seed=6)
    plain = ra.Scorer(ms, kind, max_frames=512)
    sharded = ra.Scorer(ms, kind, max_frames=512, devices=[0] * world)
    n, exchange = sharded.shard_info()
    assert n == world and exchange == "copy"
    assert parallel.split_mixtures(parallel.density_shards(ms.mixture_offsets, world)), "case must split mixtures"
    ref_s, ref_b = plain.score_host(frames)
    s, b = sharded.score_host(frames)
    _compare(kind, ms, frames, s, b, ref_s, ref_b)


@pytest.mark.gpu
def test_sharded_one_device_is_unsharded(gpu):
    ms = _ragged_model()
    frames = ra.synthetic_frames(100, 39, seed=7)
    for kind in KINDS:
        one = ra.Scorer(ms, kind, max_frames=128, devices=[0])
        assert one.shard_info() == (1, "auto")
        ref_s, ref_b = ra.Scorer(ms, kind, max_frames=128).score_host(frames)
        s, b = one.score_host(frames)
        assert np.array_equal(s.view(np.uint32), ref_s.view(np.uint32))
        if kind in ("SIMD-diagonal-maximum", "diagonal-maximum"):  # batch types write no best densities
            assert np.array_equal(b, ref_b)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["SIMD-diagonal-maximum", "diagonal-maximum"])
def test_sharded_ring_frame_major_keep_best(gpu, kind):
    ms = _ragged_model()
    ring_size, first, n = 96, 70, 80  # wrapped ring
    ring = ra.synthetic_frames(ring_size, 39, seed=8)
    sharded = ra.Scorer(ms, kind, max_frames=128, devices=[0, 0, 0])
    plain = ra.Scorer(ms, kind, max_frames=128)
    for frame_major in (False, True):
        shape = (ring_size, ms.n_mixtures) if frame_major else (ms.n_mixtures, ring_size)
        out_s, out_p = np.zeros(shape, np.float32), np.zeros(shape, np.float32)
        best_s, best_p = np.zeros(shape, np.uint32), np.zeros(shape, np.uint32)
        cid = sharded.score_host_ring(ring, first, n, out_s, keep_best=True, frame_major=frame_major)
        sharded.fetch_best(cid, best_s)
        plain.score_host_ring(ring, first, n, out_p, best_out=best_p, frame_major=frame_major)
        if kind == "SIMD-diagonal-maximum":
            assert np.array_equal(out_s.view(np.uint32), out_p.view(np.uint32))
            assert np.array_equal(best_s, best_p)
        else:
            rows = [(first + i) % ring_size for i in range(n)]
            s = out_s[rows].T if frame_major else out_s[:, rows]
            b = best_s[rows].T if frame_major else best_s[:, rows]
            frames = np.stack([ring[r] for r in rows])
            _compare(kind, ms, frames, np.ascontiguousarray(s), np.ascontiguousarray(b), None, None)


@pytest.mark.gpu
def test_sharded_score_device(gpu):
    import torch
    ms = _ragged_model()
    frames = ra.synthetic_frames(200, 39, seed=9)
    kind = "SIMD-diagonal-maximum"
    sharded = ra.Scorer(ms, kind, max_frames=256, devices=[0, 0])
    ref_s, ref_b = ra.Scorer(ms, kind, max_frames=256).score_host(frames)
    fr = torch.from_numpy(frames).to(gpu)
    s = torch.zeros((ms.n_mixtures, 200), dtype=torch.float32, device=gpu)
    b = torch.zeros((ms.n_mixtures, 200), dtype=torch.int32, device=gpu)
    for _ in range(2):  # the second call reuses the parts' buffers after the first's reads
        sharded.score_device(fr, s, b)
    torch.cuda.synchronize()
    assert np.array_equal(s.cpu().numpy().view(np.uint32), ref_s.view(np.uint32))
    assert np.array_equal(b.cpu().numpy().view(np.uint32), ref_b)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", QUANTIZED)
def test_sharded_ragged_800k_eight_parts(gpu, kind):
    """Config 4's ragged 800k-density model over 8 parts (7 split mixtures), 4096 frames in 2 host chunks."""
    counts = ra.ragged_counts(5000, 800_000, seed=99)
    ms = ra.synthetic_mixture_set(5000, counts, 39, seed=2025)
    frames = ra.synthetic_frames(2048, 39, seed=80)
    ref_s, ref_b = ra.Scorer(ms, kind, max_frames=2048).score_host(frames)
    s, b = ra.Scorer(ms, kind, max_frames=2048, devices=[0] * 8).score_host(frames)
    _compare(kind, ms, frames, s, b, ref_s, ref_b)


@pytest.mark.gpu
def test_sharded_refusals(gpu):
    ms = _ragged_model()
    for kind in ("diagonal-sum", "preselection-batch-int", "preselection-batch-float"):
        with pytest.raises(_capi.GmmError):
            ra.Scorer(ms, kind, max_frames=16, devices=[0, 0])
    # parts sharing a GPU fold their keys on it before the all-reduce: RCCL over [0, 0] is a one-rank communicator
    assert ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=16, devices=[0, 0], exchange="rccl").shard_info() == \
        (2, "rccl")
    with pytest.raises(_capi.GmmError):
        ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=16, devices=[0, 0], mixture_range=(0, 10))
    with pytest.raises(_capi.GmmError):
        ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=16, devices=[0, 0], score_scale=-1.0)


@pytest.mark.gpu
def test_bench_capi_sharded_child(gpu):
    """bench.py's N > 1 record `density_sharded_capi` (rank 0's child process over all GPUs) on one GPU: three
    parts on device 0 (copy exchange) of a ragged model, bit-exact against the unsharded scorer."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--capi-sharded-child", "0,0,0",
                        "--mixtures", "500", "--densities", "40"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["parts"] == 3 and rec["exchange"] == "copy" and rec["split_mixtures"] > 0
    assert rec["check"] == "bit-exact vs the unsharded scorer", rec


def test_sharded_create_refusals_before_any_device(built):
    """Argument checks of gmm_scorer_create_sharded that precede any HIP call (run on the CPU): unknown
    exchange, types whose split mixtures a minimum cannot combine, a mixture range, a non-positive score scale,
    no devices."""
    lib = _capi.load_library()
    ms = _ragged_model()
    desc = ms.desc()
    devs = (ctypes.c_int * 2)(0, 0)
    h = ctypes.c_void_p()

    def create(kind="SIMD-diagonal-maximum", exchange=0, n=2, **cfg_fields):
        cfg = _capi.ScorerConfig()
        lib.gmm_default_config(ctypes.byref(cfg))
        for k, v in cfg_fields.items():
            setattr(cfg, k, v)
        return lib.gmm_scorer_create_sharded(ctypes.byref(desc), _capi.SCORER_TYPES[kind], ctypes.byref(cfg), devs, n,
                                             exchange, ctypes.byref(h))

    assert create(exchange=7) == -1                                  # GMM_ERR_INVALID_ARGUMENT
    assert create(n=0) == -1
    for kind in ("diagonal-sum", "preselection-batch-int", "preselection-batch-float"):
        assert create(kind) == -2, kind                              # GMM_ERR_UNSUPPORTED
        assert b"minimum" in lib.gmm_last_error()
    assert create(mixture_begin=0, mixture_end=10) == -2
    assert create(score_scale=-1.0) == -2
    assert create(score_scale=0.0) == -2
    assert not h.value


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["SIMD-diagonal-maximum", "batch-diagonal-maximum-int"])
def test_sharded_host_pipeline_chunks(gpu, kind):
    """A host call large enough for the chunked copy-out pipeline (table >= 8 MB, >= 2 x 8192 frames): every
    frame chunk runs the whole group (parts, key exchange, assembly) before its copy-out."""
    counts = ra.ragged_counts(200, 200 * 12, low=1, high=24, seed=21)
    ms = ra.synthetic_mixture_set(200, counts, 39, seed=22, weights="random")
    frames = ra.synthetic_frames(16500, 39, seed=23)
    ref_s, ref_b = ra.Scorer(ms, kind, max_frames=16500).score_host(frames)
    s, b = ra.Scorer(ms, kind, max_frames=16500, devices=[0, 0, 0]).score_host(frames)
    assert np.array_equal(s.view(np.uint32), ref_s.view(np.uint32))
    if kind.startswith("SIMD"):
        assert np.array_equal(b, ref_b)
