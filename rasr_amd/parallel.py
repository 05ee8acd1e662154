"""Multi-GPU layouts of the scorer: one process per GPU, torch.distributed (RCCL over xGMI).

RASR itself has no in-process parallelism for scoring; its data parallelism is
corpus partitioning into independent processes (src/Bliss/CorpusDescription.cc:167-174).
Two layouts are provided:

* frame sharding ("frames", BASELINE configs 2-3): every rank holds a replica of
  the prepared model and scores its own contiguous frame range.  No collective on
  the data path; `gather_frames` exists only for callers that want the whole
  table on every rank.
* mixture sharding ("mixtures"): every rank holds the tiles of a contiguous,
  density-balanced mixture range (quantization scale computed over the whole
  model, so each shard's scores are bit-identical to the unsharded scorer) and
  scores ALL frames; the [M][F] score table is assembled with one all-gather.
  Mixture-aligned shards make the exchange a concatenation, never a min-reduce.
* density sharding ("densities", BASELINE config 4 as written): the flattened
  mixture entries are cut into P equal contiguous ranges, so a mixture on a
  boundary is split between two ranks.  Each rank scores ALL frames against its
  densities; whole mixtures are assembled by the all-gather, and the split ones
  meet in the per-frame reduce: their partial (score, best density) pairs are
  packed into order-preserving int64 keys (gmm_shard_pack_keys) and combined
  with one RCCL all-reduce(MIN) over xGMI.
"""
from __future__ import annotations

import numpy as np


def frame_shard(n_frames: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous frame range of `rank` (sizes differ by at most one)."""
    b = n_frames * rank // world
    e = n_frames * (rank + 1) // world
    return b, e


def mixture_shards(mixture_offsets, world: int) -> list[tuple[int, int]]:
    """Split mixtures into `world` contiguous ranges with about equal numbers of densities."""
    off = np.asarray(mixture_offsets, dtype=np.int64)
    m = off.shape[0] - 1
    total = int(off[-1])
    bounds = [0]
    for r in range(1, world):
        target = total * r / world
        i = int(np.searchsorted(off, target, side="left"))
        i = max(bounds[-1], min(i, m))
        bounds.append(i)
    bounds.append(m)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def _all_gather_rows(local, rows: list[int], group=None):
    """all-gather of [rows_r, ...] blocks of different heights -> concatenated table."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    hmax = max(rows)
    pad = torch.zeros((hmax,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    out = torch.empty((world * hmax,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, pad, group=group)
    parts = [out[r * hmax: r * hmax + rows[r]] for r in range(world)]
    return torch.cat(parts, dim=0)


def gather_mixture_shards(local_scores, shards, group=None):
    """Assemble the full mixture-major table [M][F] from per-rank [M_r][F] blocks."""
    return _all_gather_rows(local_scores, [e - b for b, e in shards], group)


def gather_frames(local_scores, n_frames: int, group=None):
    """Assemble [M][F] from per-rank frame ranges [M][F_r] (frame sharding)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    sizes = [frame_shard(n_frames, r, world) for r in range(world)]
    t = _all_gather_rows(local_scores.t().contiguous(), [e - b for b, e in sizes], group)
    return t.t().contiguous()


class MixtureShardedScorer:
    """Density-sharded scorer (BASELINE config 4): this rank's mixture range + all-gather."""

    def __init__(self, mixture_set, scorer_type, max_frames: int, rank: int, world: int, device: int = 0,
                 group=None, **kw):
        from .scorer import Scorer
        self.shards = mixture_shards(mixture_set.mixture_offsets, world)
        self.rank = rank
        self.group = group
        b, e = self.shards[rank]
        self.scorer = Scorer(mixture_set, scorer_type, max_frames=max_frames, device=device, mixture_range=(b, e),
                             **kw)
        self.n_local = e - b

    def score(self, frames, local_scores, local_best=None, stream=None):
        """Score all frames for this rank's mixtures and return the gathered [M][F] table."""
        self.scorer.score_device(frames, local_scores, local_best, stream)
        return gather_mixture_shards(local_scores[:, : frames.shape[0]], self.shards, self.group)


# ---------------------------------------------------------------------------
# density sharding (BASELINE config 4)
# ---------------------------------------------------------------------------
INT64_MAX = (1 << 63) - 1


def density_shards(mixture_offsets, world: int) -> list[dict]:
    """Per rank: entry range [eb, ee) = [E r / P, E (r+1) / P), the mixtures [mb, me) it scores (those with
    entries in the range; an empty mixture goes to the rank whose range holds its position), and `first_offset`,
    the in-mixture index of its first entry of mixture mb (> 0 when mb started on the previous rank)."""
    off = np.asarray(mixture_offsets, dtype=np.int64)
    m_total, e_total = off.shape[0] - 1, int(off[-1])
    ranges = [(e_total * r // world, e_total * (r + 1) // world) for r in range(world)]
    owners = [[] for _ in range(world)]
    for m in range(m_total):
        a, b = int(off[m]), int(off[m + 1])
        if a == b:  # empty: the first rank whose range reaches past its position (else the last)
            r = next((r for r, (eb, ee) in enumerate(ranges) if a < ee), world - 1)
            owners[r].append(m)
            continue
        for r, (eb, ee) in enumerate(ranges):
            if a < ee and b > eb:
                owners[r].append(m)
    out = []
    for r, (eb, ee) in enumerate(ranges):
        ms_r = owners[r]
        mb, me = (ms_r[0], ms_r[-1] + 1) if ms_r else (0, 0)
        assert me - mb == len(ms_r)
        first = max(0, eb - int(off[mb])) if ms_r else 0
        out.append({"entries": (eb, ee), "mixtures": (mb, me), "first_offset": first})
    return out


def split_mixtures(shards) -> list[int]:
    """Mixtures held by more than one rank (they need the per-frame reduce)."""
    seen, split = {}, set()
    for sh in shards:
        for m in range(*sh["mixtures"]):
            if m in seen:
                split.add(m)
            seen[m] = True
    return sorted(split)


def density_shard_model(ms, shard):
    """The mixture set rank `shard` scores: mixtures [mb, me) restricted to the entry range (same densities,
    means and covariances, so model-global preparation -- the quantization scale -- is unchanged)."""
    from .mixture_set import MixtureSet
    (eb, ee), (mb, me) = shard["entries"], shard["mixtures"]
    off = ms.mixture_offsets.astype(np.int64)
    lo = np.clip(off[mb:me + 1], eb, ee) if me > mb else np.array([eb], np.int64)
    if me > mb:
        lo[0] = max(eb, int(off[mb]))
    return MixtureSet(ms.means, ms.variances, ms.density_mean, ms.density_covariance, (lo - lo[0]).astype(np.uint32),
                      ms.mixture_densities[lo[0]:lo[-1]], ms.mixture_log_weights[lo[0]:lo[-1]])


class HipShardOps:
    """The device side of the density-sharded layout: scorers on this GPU, key packing by the library's
    kernels (gmm_shard_pack_keys / gmm_shard_unpack_keys)."""

    def __init__(self, device: int = 0):
        import torch
        self.device = torch.device("cuda", device)
        self._dev = device
        self._offsets = {}

    def scorer(self, sub_ms, scorer_type, max_frames, **kw):
        from .scorer import Scorer
        return Scorer(sub_ms, scorer_type, max_frames=max_frames, device=self._dev, **kw)

    def pack(self, scores_row, best_row, offset: int, n: int, keys_row, stream):
        import torch
        from . import _capi
        off = self._offsets.get(offset)
        if off is None:
            off = self._offsets[offset] = torch.tensor([offset], dtype=torch.int32, device=self.device)
        _capi.check(_capi.load_library().gmm_shard_pack_keys(
            scores_row.data_ptr(), None if best_row is None else best_row.data_ptr(), off.data_ptr(), 1, n,
            scores_row.shape[-1], keys_row.data_ptr(), _stream_handle(stream, self.device)), "gmm_shard_pack_keys")

    def unpack(self, keys, want_best: bool, stream):
        import torch
        from . import _capi
        rows, n = keys.shape
        s_rows = torch.empty((rows, n), dtype=torch.float32, device=keys.device)
        b_rows = torch.empty((rows, n), dtype=torch.int32, device=keys.device) if want_best else None
        _capi.check(_capi.load_library().gmm_shard_unpack_keys(
            keys.data_ptr(), rows, n, s_rows.data_ptr(), None if b_rows is None else b_rows.data_ptr(), n,
            _stream_handle(stream, self.device)), "gmm_shard_unpack_keys")
        return s_rows, b_rows


# scorer types whose mixture score is the minimum over its densities' scores (so a mixture split between
# shards is combined exactly by a per-frame minimum)
MIN_REDUCIBLE_TYPES = frozenset({"SIMD-diagonal-maximum", "diagonal-maximum", "batch-diagonal-maximum-int",
                                 "batch-diagonal-maximum-float", "batch-diagonal-maximum-fast"})


class DensityShardedScorer:
    """BASELINE config 4: this rank's equal share of the densities, all frames; whole mixtures all-gathered,
    mixtures split between ranks reduced per frame with an RCCL all-reduce(MIN) over packed keys.
    `ops` supplies the device side (HipShardOps by default)."""

    def __init__(self, mixture_set, scorer_type, max_frames: int, rank: int, world: int, device: int = 0,
                 group=None, ops=None, **kw):
        import torch
        from . import _capi
        name = scorer_type if isinstance(scorer_type, str) else next(
            (k for k, v in _capi.SCORER_TYPES.items() if v == int(scorer_type)), str(scorer_type))
        if name not in MIN_REDUCIBLE_TYPES:
            # a split mixture's parts meet in an element-wise minimum: exact for the max-approximation scorers
            # only (diagonal-sum needs a log-add of the partial sums; the preselection types cluster the
            # densities of the whole set, which a shard's sub-model would not reproduce)
            raise ValueError(f"density sharding supports {sorted(MIN_REDUCIBLE_TYPES)}, not {scorer_type!r}")
        self.ops = ops or HipShardOps(device)
        self.shards = density_shards(mixture_set.mixture_offsets, world)
        self.split = split_mixtures(self.shards)
        self.rank, self.world, self.group = rank, world, group
        self.n_mixtures = mixture_set.n_mixtures
        sh = self.shards[rank]
        self.mb, self.me = sh["mixtures"]
        self.n_local = self.me - self.mb
        self.scorer = (self.ops.scorer(density_shard_model(mixture_set, sh), scorer_type, max_frames, **kw)
                       if self.n_local > 0 else None)
        # the split mixtures this rank holds: (slot in the reduce buffer, local row, in-mixture offset of its
        # first entry -- non-zero only for the rank's first mixture when it began on the previous rank)
        self._held = [(i, m - self.mb, sh["first_offset"] if m == self.mb else 0)
                      for i, m in enumerate(self.split) if self.mb <= m < self.me]
        # rows of the all-gathered table that are a mixture's first occurrence (drops the duplicates of splits)
        rows, seen, keep = 0, set(), []
        for s_ in self.shards:
            for m in range(*s_["mixtures"]):
                if m not in seen:
                    seen.add(m)
                    keep.append(rows)
                rows += 1
        dev = self.ops.device
        self._keep = torch.tensor(keep, dtype=torch.int64, device=dev)
        self._split_idx = torch.tensor(self.split, dtype=torch.int64, device=dev)

    def partial_keys(self, local_scores, local_best, n_frames: int, stream=None):
        """int64 [len(split)][n_frames] keys of this rank's partial minima of the split mixtures (INT64_MAX where
        it holds none of a mixture)."""
        import torch
        keys = torch.full((len(self.split), n_frames), INT64_MAX, dtype=torch.int64, device=self.ops.device)
        for slot, row, offset in self._held:
            self.ops.pack(local_scores[row], None if local_best is None else local_best[row], offset, n_frames,
                          keys[slot], stream)
        return keys

    def score(self, frames, local_scores, local_best=None, stream=None):
        """Score all frames against this rank's densities; returns (scores [M][F], best [M][F] or None), the
        table of the unsharded scorer, on every rank."""
        import torch.distributed as dist
        n = frames.shape[0]
        if self.scorer is not None:
            self.scorer.score_device(frames, local_scores, local_best, stream)
        keys = self.partial_keys(local_scores, local_best, n, stream)
        if self.split:
            dist.all_reduce(keys, op=dist.ReduceOp.MIN, group=self.group)  # the per-frame reduce
        heights = [s_["mixtures"][1] - s_["mixtures"][0] for s_ in self.shards]
        full = _all_gather_rows(local_scores[: self.n_local, :n], heights, self.group).index_select(0, self._keep)
        fullb = None
        if local_best is not None:
            fullb = _all_gather_rows(local_best[: self.n_local, :n], heights, self.group).index_select(0, self._keep)
        if self.split:
            s_rows, b_rows = self.ops.unpack(keys, fullb is not None, stream)
            full[self._split_idx] = s_rows
            if fullb is not None:
                fullb[self._split_idx] = b_rows.to(fullb.dtype)
        return full, fullb


def _stream_handle(stream, device=None):
    """Raw hipStream_t for the C-ABI.  None means torch's current stream on `device` (as
    Scorer.score_device resolves it), never the legacy null stream: the key packing must be ordered
    after the scoring and before the RCCL collectives, which both run on the current stream."""
    if stream is None:
        import torch
        stream = torch.cuda.current_stream(device)
    return ctypes_stream(stream)


def ctypes_stream(stream):
    import ctypes
    h = getattr(stream, "cuda_stream", stream)
    return ctypes.c_void_p(int(h)) if h is not None else None
