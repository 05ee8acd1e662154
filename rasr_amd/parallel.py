"""Multi-GPU layouts of the scorer: one process per GPU, torch.distributed (RCCL over xGMI).

RASR itself has no in-process parallelism for scoring; its data parallelism is
corpus partitioning into independent processes (src/Bliss/CorpusDescription.cc:167-174).
Two layouts are provided:

* frame sharding ("frames", BASELINE configs 2-3): every rank holds a replica of
  the prepared model and scores its own contiguous frame range.  No collective on
  the data path; `gather_frames` exists only for callers that want the whole
  table on every rank.
* mixture sharding ("mixtures", BASELINE config 4): every rank holds the tiles of
  a contiguous, density-balanced mixture range (quantization scale computed over
  the whole model, so each shard's scores are bit-identical to the unsharded
  scorer) and scores ALL frames; the [M][F] score table is assembled with one
  all-gather.  Mixture-aligned shards make the exchange a concatenation, never a
  min-reduce.
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
