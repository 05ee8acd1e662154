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


# ---------------------------------------------------------------------------
# density sharding (BASELINE config 4): split mixtures meet in an all-reduce(MIN) over packed keys
# ---------------------------------------------------------------------------
def _pack_keys_ref(scores, best, offset):
    """The key encoding of gmm_shard_pack_keys, restated (test reference)."""
    u = scores.astype(np.float32).view(np.uint32).astype(np.uint64)
    u = np.where(u == 0x80000000, 0, u)  # -0 ties with +0, as under the reference's strict <
    o = np.where(u >= 0x80000000, u ^ 0x7FFFFFFF, u)
    d = np.zeros_like(u) if best is None else best.astype(np.uint64)
    if best is not None:
        d = np.where(d != 0xFFFFFFFF, d + offset, d)
    return ((o << np.uint64(32)) | d).view(np.int64)


def _unpack_keys_ref(keys):
    k = keys.view(np.uint64)
    o = (k >> np.uint64(32)).astype(np.uint32)
    u = np.where(o >= 0x80000000, o ^ 0x7FFFFFFF, o).astype(np.uint32)
    return u.view(np.float32), (k & np.uint64(0xFFFFFFFF)).astype(np.uint32)


class _OracleSimdShard:
    def __init__(self, sub_ms):
        self.o = oracle.OracleSimd(sub_ms)

    def score_device(self, frames, scores, best, stream=None):
        s, b, _ = self.o.score(frames.numpy())
        scores[: s.shape[0], : s.shape[1]] = torch.from_numpy(s)
        if best is not None:
            best[: b.shape[0], : b.shape[1]] = torch.from_numpy(b.view(np.int32))


class _NumpyShardOps:
    """CPU stand-in for HipShardOps in the gloo test: oracle scorer, numpy key encoding."""
    device = torch.device("cpu")

    def scorer(self, sub_ms, scorer_type, max_frames, **kw):
        return _OracleSimdShard(sub_ms)

    def pack(self, scores_row, best_row, offset, n, keys_row, stream):
        b = None if best_row is None else best_row[:n].numpy().view(np.uint32)
        keys_row[:n] = torch.from_numpy(_pack_keys_ref(scores_row[:n].numpy(), b, offset))

    def unpack(self, keys, want_best, stream):
        s, b = _unpack_keys_ref(keys.numpy())
        return torch.from_numpy(s.copy()), (torch.from_numpy(b.view(np.int32).copy()) if want_best else None)


DENSITY_COUNTS = [3, 9, 1, 16, 17, 2, 5, 8, 30, 4, 4, 6, 7, 1, 1, 12, 3, 9, 2, 40, 11, 5, 6]


def _density_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ms = ra.synthetic_mixture_set(23, DENSITY_COUNTS, 39, seed=33, weights="random")
        frames = torch.from_numpy(ra.synthetic_frames(29, 39, seed=34))
        sc = parallel.DensityShardedScorer(ms, "SIMD-diagonal-maximum", 29, rank, world, ops=_NumpyShardOps())
        local_s = torch.zeros((max(sc.n_local, 1), 29), dtype=torch.float32)
        local_b = torch.zeros((max(sc.n_local, 1), 29), dtype=torch.int32)
        full, fullb = sc.score(frames, local_s, local_b)
        q.put((rank, full.numpy(), fullb.numpy(), sc.split))
    finally:
        dist.destroy_process_group()


def test_density_shards_plan():
    off = np.cumsum([0] + DENSITY_COUNTS)
    for world in (1, 2, 3, 5, 8, 300):
        sh = parallel.density_shards(off, world)
        # every entry scored exactly once, every mixture by >= 1 rank, ranges contiguous in mixtures
        assert sum(s["entries"][1] - s["entries"][0] for s in sh) == off[-1]
        held = sorted({m for s in sh for m in range(*s["mixtures"])})
        assert held == list(range(len(DENSITY_COUNTS)))
        ms = ra.synthetic_mixture_set(23, DENSITY_COUNTS, 8, seed=1)
        for s in sh:
            sub = parallel.density_shard_model(ms, s)
            assert sub.n_entries == s["entries"][1] - s["entries"][0]
            assert sub.n_mixtures == s["mixtures"][1] - s["mixtures"][0]


def test_shard_key_encoding_orders_like_the_reference():
    rng = np.random.default_rng(5)
    s = np.concatenate([rng.standard_normal(500).astype(np.float32) * 100, np.array([0.0, -0.0, 1e30, -1e30],
                                                                                       np.float32)])
    b = rng.integers(0, 1000, s.shape[0]).astype(np.uint32)
    k = _pack_keys_ref(s, b, 0)
    order = np.argsort(k, kind="stable")
    ref = np.lexsort((b, s))  # by score, then density
    assert np.array_equal(s[order], s[ref]) and np.array_equal(b[order], b[ref])
    s2, b2 = _unpack_keys_ref(k)
    assert np.array_equal(s2, s) and np.array_equal(b2, b)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_gloo_density_sharded_min_reduce(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_density_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ms = ra.synthetic_mixture_set(23, DENSITY_COUNTS, 39, seed=33, weights="random")
    want_s, want_b, _ = oracle.OracleSimd(ms).score(ra.synthetic_frames(29, 39, seed=34))
    for _, full, fullb, split in res:
        assert split, "the case must split mixtures between ranks"
        assert np.array_equal(full.view(np.uint32), want_s.view(np.uint32))
        assert np.array_equal(fullb.view(np.uint32), want_b)
