"""N>1 layouts on CPU with the gloo backend (world_size 2, 127.0.0.1).

The device compute is replaced by the oracle's per-shard scores (the GPU kernels
are covered by the gpu tests); what is tested here is the sharding arithmetic and
the collective that assembles the score table."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
import rasr_amd as ra
from rasr_amd import parallel


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_model(ms, b, e):
    """The sub-mixture-set of mixtures [b, e) (same densities, means, covariances)."""
    o = ms.mixture_offsets
    off = (o[b: e + 1] - o[b]).astype(np.uint32)
    return ra.MixtureSet(ms.means, ms.variances, ms.density_mean, ms.density_covariance, off,
                         ms.mixture_densities[o[b]: o[e]], ms.mixture_log_weights[o[b]: o[e]])


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ms = ra.synthetic_mixture_set(23, [3, 9, 1, 16, 17, 2, 5, 8, 30, 4, 4, 6, 7, 1, 1, 12, 3, 9, 2, 40, 11, 5, 6],
                                      39, seed=31, weights="random")
        frames = ra.synthetic_frames(37, 39, seed=32)
        # mixture sharding: float scorer restated per shard, gathered
        shards = parallel.mixture_shards(ms.mixture_offsets, world)
        b, e = shards[rank]
        local = oracle.OracleFloat(_shard_model(ms, b, e)).score(frames)[0]
        full = parallel.gather_mixture_shards(torch.from_numpy(local), shards)
        # frame sharding: each rank scores its frame range, gathered along frames
        fb, fe = parallel.frame_shard(len(frames), rank, world)
        lf = oracle.OracleSimd(ms).score(frames[fb:fe])[0]
        fullf = parallel.gather_frames(torch.from_numpy(lf), len(frames))
        q.put((rank, full.numpy(), fullf.numpy()))
    finally:
        dist.destroy_process_group()


def test_mixture_shards_balanced():
    off = np.cumsum([0] + [160] * 5000)
    sh = parallel.mixture_shards(off, 8)
    assert sh[0][0] == 0 and sh[-1][1] == 5000
    assert all(a[1] == b[0] for a, b in zip(sh[:-1], sh[1:]))
    sizes = [off[e] - off[b] for b, e in sh]
    assert max(sizes) - min(sizes) <= 160
    assert parallel.frame_shard(10, 0, 3) == (0, 3) and parallel.frame_shard(10, 2, 3) == (6, 10)


def test_float_scores_of_a_shard_equal_the_full_model():
    # the float scorer has no model-global state, so the shard model restates the shard exactly
    ms = ra.synthetic_mixture_set(10, 7, 39, seed=3)
    fr = ra.synthetic_frames(9, 39, seed=4)
    full = oracle.OracleFloat(ms).score(fr)[0]
    assert np.array_equal(oracle.OracleFloat(_shard_model(ms, 3, 8)).score(fr)[0], full[3:8])


@pytest.mark.timeout(300)
def test_gloo_world2_gathers():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ms = ra.synthetic_mixture_set(23, [3, 9, 1, 16, 17, 2, 5, 8, 30, 4, 4, 6, 7, 1, 1, 12, 3, 9, 2, 40, 11, 5, 6],
                                  39, seed=31, weights="random")
    frames = ra.synthetic_frames(37, 39, seed=32)
    want = oracle.OracleFloat(ms).score(frames)[0]
    wantf = oracle.OracleSimd(ms).score(frames)[0]
    for _, full, fullf in res:
        assert np.array_equal(full, want)
        assert np.array_equal(fullf.view(np.uint32), wantf.view(np.uint32))
