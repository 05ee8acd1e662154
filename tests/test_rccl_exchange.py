"""The RCCL exchange of the density-sharded layout, executed on one GPU.

gmm_scorer_create_sharded's RCCL exchange (gmm_api.cc groupScore) folds the keys of the parts that share a GPU
into that GPU's first part (minIntoShardKeys) and then all-reduces (ncclMin, ncclInt64, in place) over one rank
per distinct GPU.  With every part on device 0 this is a ONE-rank communicator (ncclCommInitAll over [0]) and the
very ncclGroupStart / ncclAllReduce / ncclGroupEnd sequence an 8-GPU handle issues -- the path a one-GPU box can
run.  It must give the same tables, bit for bit, as the copy exchange (peer copies + minShardKeys) that the other
sharded tests check against the unsharded scorer and the oracle.

What only an 8-GPU run exercises: ranks on distinct devices (the all-reduce moving data over xGMI), the
cross-device stream waits on the lead's start event, and the peer copies of frames and tables (DESIGN.md
section 5).

The torch side (rasr_amd/parallel.py DensityShardedScorer, what bench.py --gpus N uses) runs over the `nccl`
(= RCCL) backend at world size 1 in a child process (tests/nccl_world1_child.py).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import rasr_amd as ra
from rasr_amd import parallel

pytestmark = pytest.mark.gpu

KINDS = ["SIMD-diagonal-maximum", "batch-diagonal-maximum-int", "diagonal-maximum", "batch-diagonal-maximum-float"]


def _ragged_model(n_mix=60, total=60 * 14, seed=5):
    counts = ra.ragged_counts(n_mix, total, low=1, high=40, seed=3)
    return ra.synthetic_mixture_set(n_mix, counts, 39, seed=seed, weights="random")


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("kind", KINDS)
def test_rccl_one_rank_equals_copy_exchange(gpu, kind, world):
    ms = _ragged_model()
    frames = ra.synthetic_frames(300, 39, seed=6)
    assert parallel.split_mixtures(parallel.density_shards(ms.mixture_offsets, world)), "case must split mixtures"
    copy = ra.Scorer(ms, kind, max_frames=512, devices=[0] * world, exchange="copy")
    rccl = ra.Scorer(ms, kind, max_frames=512, devices=[0] * world, exchange="rccl")
    assert rccl.shard_info() == (world, "rccl")
    s_c, b_c = copy.score_host(frames)
    for _ in range(2):  # the second call reuses the keys buffers after the first call's all-reduce
        s_r, b_r = rccl.score_host(frames)
        assert np.array_equal(_bits(s_r), _bits(s_c))
        if kind in ("SIMD-diagonal-maximum", "diagonal-maximum"):
            assert np.array_equal(b_r, b_c)
    if kind in ("SIMD-diagonal-maximum", "batch-diagonal-maximum-int"):  # and the unsharded scorer, bit for bit
        ref_s, ref_b = ra.Scorer(ms, kind, max_frames=512).score_host(frames)
        assert np.array_equal(_bits(s_r), _bits(ref_s))
        if kind == "SIMD-diagonal-maximum":
            assert np.array_equal(b_r, ref_b)


def test_rccl_one_rank_device_and_ring(gpu):
    import torch
    ms = _ragged_model()
    kind = "SIMD-diagonal-maximum"
    frames = ra.synthetic_frames(200, 39, seed=9)
    ref_s, ref_b = ra.Scorer(ms, kind, max_frames=256).score_host(frames)
    sc = ra.Scorer(ms, kind, max_frames=256, devices=[0, 0, 0], exchange="rccl")
    fr = torch.from_numpy(frames).to(gpu)
    s = torch.zeros((ms.n_mixtures, 200), dtype=torch.float32, device=gpu)
    b = torch.zeros((ms.n_mixtures, 200), dtype=torch.int32, device=gpu)
    for _ in range(3):  # back-to-back calls on one stream, no host sync between them
        sc.score_device(fr, s, b)
    torch.cuda.synchronize()
    assert np.array_equal(_bits(s.cpu().numpy()), _bits(ref_s))
    assert np.array_equal(b.cpu().numpy().view(np.uint32), ref_b)
    # the ring protocol with kept best densities (the C++ drop-in's calls)
    ring_size, first, n = 96, 70, 80
    ring = ra.synthetic_frames(ring_size, 39, seed=8)
    plain = ra.Scorer(ms, kind, max_frames=128)
    sc2 = ra.Scorer(ms, kind, max_frames=128, devices=[0, 0, 0], exchange="rccl")
    for frame_major in (False, True):
        shape = (ring_size, ms.n_mixtures) if frame_major else (ms.n_mixtures, ring_size)
        out_s, out_p = np.zeros(shape, np.float32), np.zeros(shape, np.float32)
        best_s, best_p = np.zeros(shape, np.uint32), np.zeros(shape, np.uint32)
        cid = sc2.score_host_ring(ring, first, n, out_s, keep_best=True, frame_major=frame_major)
        sc2.fetch_best(cid, best_s)
        plain.score_host_ring(ring, first, n, out_p, best_out=best_p, frame_major=frame_major)
        assert np.array_equal(_bits(out_s), _bits(out_p))
        assert np.array_equal(best_s, best_p)


@pytest.mark.parametrize("kind", ["SIMD-diagonal-maximum", "batch-diagonal-maximum-int"])
def test_rccl_one_rank_800k_eight_parts(gpu, kind):
    """Config 4's ragged 800k-density model, 8 parts (7 split mixtures) folded on one GPU + a one-rank all-reduce."""
    counts = ra.ragged_counts(5000, 800_000, seed=99)
    ms = ra.synthetic_mixture_set(5000, counts, 39, seed=2025)
    frames = ra.synthetic_frames(2048, 39, seed=80)
    ref_s, ref_b = ra.Scorer(ms, kind, max_frames=2048).score_host(frames)
    s, b = ra.Scorer(ms, kind, max_frames=2048, devices=[0] * 8, exchange="rccl").score_host(frames)
    assert np.array_equal(_bits(s), _bits(ref_s))
    if kind.startswith("SIMD"):
        assert np.array_equal(b, ref_b)


@pytest.mark.timeout(300)
def test_torch_nccl_world1_density_sharded(gpu):
    """DensityShardedScorer over torch.distributed's nccl (RCCL) backend at world size 1, and an int64 MIN
    all-reduce of shard keys on that backend (the dtype and op the per-frame reduce needs)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "nccl_world1_child.py")], capture_output=True,
                       text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["backend"] == "nccl" and rec["world"] == 1, rec
    assert rec["scores"] == "bit-exact vs the unsharded scorer" and rec["best"] == "equal", rec
    assert rec["all_reduce_min_int64"] == "ok", rec
