"""Density-sharded layout (BASELINE config 4) on one GPU: the shards of P virtual ranks are scored by
the real kernels, their split mixtures packed by gmm_shard_pack_keys, combined by the element-wise
minimum an RCCL all-reduce(MIN) computes, unpacked by gmm_shard_unpack_keys, and the table compared
with the unsharded scorer: bit-exact (scores and best densities) for the quantized types, within the
float contract (1e-4 relative) for diagonal-maximum.  The collectives themselves run in
tests/test_distributed.py (gloo, world 2 and 3)."""
import numpy as np
import pytest
import torch

import rasr_amd as ra
from rasr_amd import parallel

pytestmark = pytest.mark.gpu


def _emulate(ms, kind, frames, world, with_best):
    dev = torch.device("cuda", 0)
    n = frames.shape[0]
    fr = torch.from_numpy(frames).to(dev)
    shards = [parallel.DensityShardedScorer(ms, kind, n, r, world, device=0) for r in range(world)]
    keys, tables, btables = None, [], []
    for sc in shards:
        ls = torch.zeros((max(sc.n_local, 1), n), dtype=torch.float32, device=dev)
        lb = torch.zeros((max(sc.n_local, 1), n), dtype=torch.int32, device=dev) if with_best else None
        if sc.scorer is not None:
            sc.scorer.score_device(fr, ls, lb)
        k = sc.partial_keys(ls, lb, n)
        keys = k if keys is None else torch.minimum(keys, k)  # = all_reduce(MIN)
        tables.append(ls[: sc.n_local])
        if with_best:
            btables.append(lb[: sc.n_local])
    sc0 = shards[0]
    full = torch.cat(tables).index_select(0, sc0._keep)  # = the all-gather, duplicates dropped
    fullb = torch.cat(btables).index_select(0, sc0._keep) if with_best else None
    if sc0.split:
        s_rows, b_rows = sc0.ops.unpack(keys, with_best, None)
        full[sc0._split_idx] = s_rows
        if with_best:
            fullb[sc0._split_idx] = b_rows
    torch.cuda.synchronize()
    return full.cpu().numpy(), (fullb.cpu().numpy().view(np.uint32) if with_best else None), sc0.split


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("kind", ["SIMD-diagonal-maximum", "batch-diagonal-maximum-int", "diagonal-maximum"])
def test_density_sharded_equals_unsharded(gpu, kind, world):
    counts = ra.ragged_counts(60, 60 * 14, low=1, high=40, seed=3)
    ms = ra.synthetic_mixture_set(60, counts, 39, seed=5, weights="random")
    frames = ra.synthetic_frames(300, 39, seed=6)
    with_best = kind != "batch-diagonal-maximum-int"
    s, b, split = _emulate(ms, kind, frames, world, with_best)
    assert split, "the case must split mixtures between shards"
    ref_s, ref_b = ra.Scorer(ms, kind, max_frames=300).score_host(frames)
    if kind == "diagonal-maximum":
        err = np.abs(s.astype(np.float64) - ref_s) / np.maximum(1.0, np.abs(ref_s.astype(np.float64)))
        assert err.max() <= 1e-4
        # best densities agree wherever the two best candidates are apart (they are on this model)
        assert (b == ref_b.view(np.uint32)).mean() > 0.999
    else:
        assert np.array_equal(s.view(np.uint32), ref_s.view(np.uint32))
        if with_best:
            assert np.array_equal(b, ref_b.view(np.uint32))


def test_shard_keys_roundtrip(gpu):
    from rasr_amd import _capi
    lib = _capi.load_library()
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(1)
    s = torch.from_numpy((rng.standard_normal((7, 33)) * 50).astype(np.float32)).to(dev)
    b = torch.from_numpy(rng.integers(0, 500, (7, 33)).astype(np.int32)).to(dev)
    off = torch.arange(7, dtype=torch.int32, device=dev) * 1000
    k = torch.empty((7, 33), dtype=torch.int64, device=dev)
    _capi.check(lib.gmm_shard_pack_keys(s.data_ptr(), b.data_ptr(), off.data_ptr(), 7, 33, 33, k.data_ptr(), None))
    s2 = torch.empty_like(s)
    b2 = torch.empty_like(b)
    _capi.check(lib.gmm_shard_unpack_keys(k.data_ptr(), 7, 33, s2.data_ptr(), b2.data_ptr(), 33, None))
    torch.cuda.synchronize()
    assert torch.equal(s2, s)
    assert torch.equal(b2, b + off[:, None])
    # signed key order = (score, density) order
    kk = k.cpu().numpy().ravel()
    ss, bb = s.cpu().numpy().ravel(), (b + off[:, None]).cpu().numpy().ravel()
    o = np.argsort(kk, kind="stable")
    r = np.lexsort((bb, ss))
    assert np.array_equal(ss[o], ss[r]) and np.array_equal(bb[o], bb[r])
