"""Python handle over the C-ABI scorer (include/rasr_gmm.h).

Used by the tests and bench.py; RASR itself binds the C-ABI from C++
(rasr_amd/csrc/host/GpuFeatureScorer.hh).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _capi
from .mixture_set import MixtureSet


def _type_id(t) -> int:
    if isinstance(t, str):
        return _capi.SCORER_TYPES[t]
    return int(t)


def default_config() -> _capi.ScorerConfig:
    cfg = _capi.ScorerConfig()
    _capi.load_library().gmm_default_config(ctypes.byref(cfg))
    return cfg


class Scorer:
    """One prepared model resident on one GPU (gmm_scorer_create), or -- with `devices` -- the density-sharded
    handle over several (gmm_scorer_create_sharded: part r of the density shard plan on devices[r], the full
    table assembled on devices[0], `exchange` "auto" / "rccl" / "copy" for the per-frame reduce)."""

    def __init__(self, mixture_set: MixtureSet, scorer_type="SIMD-diagonal-maximum", max_frames: int = 4096,
                 device: int = 0, mixture_weight_scale: float = 1.0, gaussian_scale: float = 1.0,
                 score_scale: float = 1.0, mixture_range: tuple[int, int] | None = None, native_f32: bool = False,
                 split_tile16: bool = False, split_tile32: bool = False, clusters: int = 256,
                 select_clusters: int = 32, clustering_iterations: int = 5, backoff_score: float = 40000.0,
                 reference_order: bool = False, devices=None, exchange: str = "auto", full_keys: bool = False,
                 no_score_only_twin: bool = False, cache_archive: str | None = None,
                 cache_archive_read_only: bool = False):
        self._lib = _capi.load_library()
        self.mixture_set = mixture_set
        self.type = _type_id(scorer_type)
        cfg = default_config()
        cfg.max_frames = int(max_frames)
        cfg.mixture_weight_scale = mixture_weight_scale
        cfg.gaussian_scale = gaussian_scale
        cfg.score_scale = score_scale
        if native_f32:  # float types: the f32-MFMA kernel instead of the split-f16 one
            cfg.flags |= _capi.GMM_FLAG_NATIVE_F32
        if split_tile16:  # split-f16 kernel: force 16-density tiles
            cfg.flags |= _capi.GMM_FLAG_SPLIT_TILE16
        if split_tile32:  # split-f16 kernel: force 32-density tiles (mixtures <= 512 densities, D <= 51)
            cfg.flags |= _capi.GMM_FLAG_SPLIT_TILE32
        if reference_order:  # float types: the reference's own f32 operation order (bit-identical, VALU rate)
            cfg.flags |= _capi.GMM_FLAG_REFERENCE_ORDER
        if full_keys:  # batch-int / -fast: the (score, density) key layout instead of the score-only one
            cfg.flags |= _capi.GMM_FLAG_FULL_KEYS
        if no_score_only_twin:  # SIMD: serve calls without best densities from the key layout too
            cfg.flags |= _capi.GMM_FLAG_NO_SCORE_ONLY_TWIN
        # density preselection ("density-clustering" parameters, preselection-batch-* types)
        cfg.clusters = int(clusters)
        cfg.select_clusters = int(select_clusters)
        cfg.clustering_iterations = int(clustering_iterations)
        cfg.backoff_score = float(backoff_score)
        # the "density-clustering" item of this RASR cache archive is read if it matches, else built and written
        self._cache_archive = None if cache_archive is None else os.fsencode(cache_archive)
        cfg.cache_archive = self._cache_archive
        if cache_archive_read_only:
            cfg.flags |= _capi.GMM_FLAG_CACHE_ARCHIVE_READ_ONLY
        if mixture_range is not None:
            cfg.mixture_begin, cfg.mixture_end = int(mixture_range[0]), int(mixture_range[1])
        self.max_frames = int(max_frames)
        self._desc = mixture_set.desc()
        h = ctypes.c_void_p()
        if devices is None:
            _capi.check(self._lib.gmm_scorer_create(ctypes.byref(self._desc), self.type, ctypes.byref(cfg),
                                                    int(device), ctypes.byref(h)), "gmm_scorer_create")
        else:
            devs = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
            _capi.check(self._lib.gmm_scorer_create_sharded(ctypes.byref(self._desc), self.type, ctypes.byref(cfg),
                                                            devs, len(devices), _capi.GMM_EXCHANGE[exchange],
                                                            ctypes.byref(h)), "gmm_scorer_create_sharded")
            device = int(devices[0])
        self._h = h
        self.device = device

    def shard_info(self) -> tuple[int, str]:
        """(parts, exchange) of the handle: (1, "auto") unsharded."""
        n, x = ctypes.c_uint32(), ctypes.c_int()
        _capi.check(self._lib.gmm_scorer_shard_info(self._h, ctypes.byref(n), ctypes.byref(x)), "gmm_scorer_shard_info")
        return n.value, {v: k for k, v in _capi.GMM_EXCHANGE.items()}[x.value]

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.gmm_scorer_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def main_kernel(self) -> str:
        """Name of the dominant kernel a score call launches (gmm_scorer_launch_info)."""
        n = ctypes.c_uint32()
        name = ctypes.c_char_p()
        _capi.check(self._lib.gmm_scorer_launch_info(self._h, 1, ctypes.byref(n), ctypes.byref(name)),
                    "gmm_scorer_launch_info")
        return name.value.decode()

    def density_clustering(self):
        """(cluster_of_entry [entries] u8, cluster_means [clusters][Dp] f32 or u8) of a preselection type."""
        n = ctypes.c_uint32()
        dp = ctypes.c_uint32()
        _capi.check(self._lib.gmm_scorer_density_clustering(self._h, ctypes.byref(n), ctypes.byref(dp), None, None),
                    "gmm_scorer_density_clustering")
        entries = int(self.mixture_set.mixture_offsets[-1])
        coe = np.zeros(entries, np.uint8)
        dtype = np.uint8 if self.type == _capi.BATCH_PRESELECTION_INT else np.float32
        means = np.zeros((n.value, dp.value), dtype)
        _capi.check(self._lib.gmm_scorer_density_clustering(self._h, None, None, coe.ctypes.data_as(ctypes.c_void_p),
                                                            means.ctypes.data_as(ctypes.c_void_p)),
                    "gmm_scorer_density_clustering")
        return coe, means

    def clustering_source(self) -> str:
        """Where the density clustering came from: "built", "written" (built and written to the cache archive) or
        "cached" (read from it); gmm_scorer_clustering_source."""
        v = ctypes.c_int()
        _capi.check(self._lib.gmm_scorer_clustering_source(self._h, ctypes.byref(v)), "gmm_scorer_clustering_source")
        return _capi.GMM_CLUSTERING[v.value]

    def cluster_selection(self, n_frames: int) -> np.ndarray:
        """The [n_frames][clusters] 0/1 selection of the last score call (synchronizes)."""
        n = ctypes.c_uint32()
        _capi.check(self._lib.gmm_scorer_density_clustering(self._h, ctypes.byref(n), None, None, None),
                    "gmm_scorer_density_clustering")
        sel = np.zeros((int(n_frames), n.value), np.uint8)
        _capi.check(self._lib.gmm_scorer_cluster_selection(self._h, int(n_frames), sel.ctypes.data_as(ctypes.c_void_p)),
                    "gmm_scorer_cluster_selection")
        return sel

    def n_mixtures(self) -> int:
        return int(self._lib.gmm_scorer_n_mixtures(self._h))

    def dimension(self) -> int:
        return int(self._lib.gmm_scorer_dimension(self._h))

    def score_device(self, frames, scores, best=None, stream=None, n_frames=None) -> None:
        """frames: torch cuda f32 [F, >=D] (row stride = frames.stride(0)); scores: [M, >=F] f32;
        best: [M, >=F] int32/uint32 or None.  Asynchronous on `stream` (torch stream or raw handle)."""
        f = int(frames.shape[0] if n_frames is None else n_frames)
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(frames.device)
        s = getattr(stream, "cuda_stream", stream)
        rc = self._lib.gmm_score_device(self._h, ctypes.c_void_p(frames.data_ptr()), f, int(frames.stride(0)),
                                        ctypes.c_void_p(scores.data_ptr()),
                                        ctypes.c_void_p(best.data_ptr()) if best is not None else None,
                                        int(scores.stride(0)), ctypes.c_void_p(s) if s else None)
        _capi.check(rc, "gmm_score_device")

    def score_host(self, frames: np.ndarray, want_best: bool = True, out: np.ndarray | None = None,
                   best_out: np.ndarray | None = None):
        """gmm_score_host.  out / best_out: caller-kept [n_mixtures][>= n_frames] tables (row stride =
        their second dimension), e.g. from pinned_empty() so the table is written by DMA directly."""
        frames = np.ascontiguousarray(frames, dtype=np.float32)
        f = frames.shape[0]
        m = self.n_mixtures()
        scores = np.empty((m, f), dtype=np.float32) if out is None else out
        best = (np.empty((m, f), dtype=np.uint32) if best_out is None else best_out) if want_best else None
        stride = scores.shape[1] if scores.ndim == 2 else f
        for name, a, dt in (("out", scores, np.float32), ("best_out", best, np.uint32)):
            if a is not None and (a.dtype != dt or a.shape != (m, stride) or not a.flags.c_contiguous or stride < f):
                raise ValueError(f"{name} must be a C-contiguous {np.dtype(dt).name} [{m}][>= {f}] array")
        rc = self._lib.gmm_score_host(self._h, frames.ctypes.data_as(ctypes.c_void_p), f, frames.shape[1],
                                      scores.ctypes.data_as(ctypes.c_void_p),
                                      best.ctypes.data_as(ctypes.c_void_p) if best is not None else None, stride)
        _capi.check(rc, "gmm_score_host")
        return scores, best

    def score_host_ring(self, ring: np.ndarray, first: int, n_frames: int, out: np.ndarray,
                        best_out: np.ndarray | None = None, keep_best: bool = False, frame_major: bool = False,
                        lazy_best: bool = False, asynchronous: bool = False) -> int:
        """gmm_score_host_ring: frames ring[(first + i) % R], i < n_frames (R = ring.shape[0]) into the ring
        positions of out / best_out: columns of [n_mixtures][>= R] tables, or with frame_major rows of
        [>= R][>= n_mixtures] tables.  keep_best: best densities stay on the device for fetch_best();
        lazy_best: scores only, fetch_best() computes the best densities from the frames kept on the device.
        asynchronous (GMM_HOST_ASYNC, page-locked tables only): returns once enqueued; wait(call id) before
        reading the tables or changing the ring rows.  Returns the call id."""
        ring = np.ascontiguousarray(ring, dtype=np.float32)
        m, R = self.n_mixtures(), ring.shape[0]
        for name, a, dt in (("out", out, np.float32), ("best_out", best_out, np.uint32)):
            if a is None:
                continue
            ok = a.dtype == dt and a.ndim == 2 and a.flags.c_contiguous and (
                (a.shape[0] >= R and a.shape[1] >= m) if frame_major else (a.shape[0] == m and a.shape[1] >= R))
            if not ok:
                raise ValueError(f"{name} must be a C-contiguous {np.dtype(dt).name} table of the ring's layout")
        if best_out is not None and best_out.shape[1] != out.shape[1]:
            raise ValueError("out and best_out must have the same row stride")
        cid = ctypes.c_uint64()
        flags = ((_capi.GMM_HOST_KEEP_BEST if keep_best else 0) | (_capi.GMM_HOST_FRAME_MAJOR if frame_major else 0) |
                 (_capi.GMM_HOST_LAZY_BEST if lazy_best else 0) | (_capi.GMM_HOST_ASYNC if asynchronous else 0))
        rc = self._lib.gmm_score_host_ring(
            self._h, ring.ctypes.data_as(ctypes.c_void_p), R, int(first), int(n_frames), ring.shape[1],
            out.ctypes.data_as(ctypes.c_void_p), best_out.ctypes.data_as(ctypes.c_void_p) if best_out is not None else None,
            out.shape[1], flags, ctypes.byref(cid))
        _capi.check(rc, "gmm_score_host_ring")
        return cid.value

    def wait(self, call_id: int) -> None:
        """gmm_host_call_wait: the GMM_HOST_ASYNC call `call_id` has written its tables."""
        _capi.check(self._lib.gmm_host_call_wait(self._h, int(call_id)), "gmm_host_call_wait")

    def fetch_best(self, call_id: int, best_out: np.ndarray) -> None:
        """gmm_fetch_best_density into the same ring columns the call's scores went to."""
        if best_out.dtype != np.uint32 or best_out.ndim != 2 or not best_out.flags.c_contiguous:
            raise ValueError("best_out must be a C-contiguous uint32 table of the call's layout")
        _capi.check(self._lib.gmm_fetch_best_density(self._h, int(call_id), best_out.ctypes.data_as(ctypes.c_void_p),
                                                     best_out.shape[1]), "gmm_fetch_best_density")

    def best_pairs(self, call_id: int, positions, mixtures) -> np.ndarray:
        """gmm_best_density_pairs: best densities of (ring position, mixture) pairs of host call `call_id` (made with
        keep_best or lazy_best), from its frames still on the device."""
        pos = np.ascontiguousarray(positions, dtype=np.uint32)
        mix = np.ascontiguousarray(mixtures, dtype=np.uint32)
        if pos.shape != mix.shape or pos.ndim != 1:
            raise ValueError("positions and mixtures must be 1-d arrays of one length")
        out = np.empty(pos.shape[0], dtype=np.uint32)
        _capi.check(self._lib.gmm_best_density_pairs(self._h, int(call_id), pos.ctypes.data_as(ctypes.c_void_p),
                                                     mix.ctypes.data_as(ctypes.c_void_p), pos.shape[0],
                                                     out.ctypes.data_as(ctypes.c_void_p)), "gmm_best_density_pairs")
        return out

    def best_pairs_device(self, frames, pair_frame, pair_mixture, out, stream=None, n_frames=None) -> None:
        """gmm_best_density_pairs_device: frames torch cuda f32 [F, >=D]; pair_frame / pair_mixture / out: int32 or
        uint32 cuda tensors of n_pairs.  Asynchronous on `stream`."""
        f = int(frames.shape[0] if n_frames is None else n_frames)
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(frames.device)
        s = getattr(stream, "cuda_stream", stream)
        n = int(pair_frame.numel())
        if pair_mixture.numel() != n or out.numel() < n:
            raise ValueError("pair_frame, pair_mixture and out must hold n_pairs entries")
        rc = self._lib.gmm_best_density_pairs_device(self._h, ctypes.c_void_p(frames.data_ptr()), f, int(frames.stride(0)),
                                                     ctypes.c_void_p(pair_frame.data_ptr()),
                                                     ctypes.c_void_p(pair_mixture.data_ptr()), n,
                                                     ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(s) if s else None)
        _capi.check(rc, "gmm_best_density_pairs_device")

    def set_timing(self, enable: bool) -> None:
        _capi.check(self._lib.gmm_scorer_set_timing(self._h, int(bool(enable))), "gmm_scorer_set_timing")

    def kernel_time(self, reset: bool = True):
        """(total ms, launches) of the scorer kernel since the last reset (HIP events on its stream)."""
        ms, n = ctypes.c_double(), ctypes.c_uint32()
        _capi.check(self._lib.gmm_scorer_kernel_time(self._h, ctypes.byref(ms), ctypes.byref(n), int(reset)),
                    "gmm_scorer_kernel_time")
        return ms.value, n.value

    def quantization(self):
        s, q = ctypes.c_float(), ctypes.c_float()
        _capi.check(self._lib.gmm_scorer_quantization(self._h, ctypes.byref(s), ctypes.byref(q)),
                    "gmm_scorer_quantization")
        return s.value, q.value

    def multiply_and_quantize(self, feature: np.ndarray) -> np.ndarray:
        feature = np.ascontiguousarray(feature, dtype=np.float32)
        dp = (self.dimension() + 15) // 16 * 16
        out = np.empty((self.mixture_set.n_covariances, dp), dtype=np.uint8)
        _capi.check(self._lib.gmm_scorer_multiply_and_quantize(self._h, feature.ctypes.data_as(ctypes.c_void_p),
                                                               out.ctypes.data_as(ctypes.c_void_p)),
                    "gmm_scorer_multiply_and_quantize")
        return out


def cache_archive_read(path: str, name: str) -> bytes:
    """Item `name` of a RASR cache archive (Core::MappedArchive layout; gmm_cache_archive_read_item)."""
    lib = _capi.load_library()
    size = ctypes.c_uint64()
    _capi.check(lib.gmm_cache_archive_read_item(os.fsencode(path), name.encode(), None, 0, ctypes.byref(size)),
                "gmm_cache_archive_read_item")
    buf = ctypes.create_string_buffer(max(size.value, 1))
    _capi.check(lib.gmm_cache_archive_read_item(os.fsencode(path), name.encode(), buf, size.value, ctypes.byref(size)),
                "gmm_cache_archive_read_item")
    return buf.raw[:size.value]


def cache_archive_write(path: str, name: str, data: bytes) -> None:
    """Write item `name` (the archive is created, or rewritten with its other items kept)."""
    lib = _capi.load_library()
    _capi.check(lib.gmm_cache_archive_write_item(os.fsencode(path), name.encode(), data, len(data)),
                "gmm_cache_archive_write_item")


def pinned_empty(shape, dtype=np.float32) -> np.ndarray:
    """Uninitialised numpy array in page-locked host memory (gmm_host_alloc; freed with the array)."""
    import weakref

    lib = _capi.load_library()
    dtype = np.dtype(dtype)
    n = int(np.prod(shape)) * dtype.itemsize
    ptr = ctypes.c_void_p()
    _capi.check(lib.gmm_host_alloc(max(n, 1), ctypes.byref(ptr)), "gmm_host_alloc")
    holder = (ctypes.c_char * max(n, 1)).from_address(ptr.value)
    weakref.finalize(holder, lib.gmm_host_free, ptr.value)
    return np.frombuffer(holder, dtype=dtype, count=int(np.prod(shape))).reshape(shape)


def prepare_quantized_host(ms: MixtureSet, scorer_type="SIMD-diagonal-maximum") -> dict:
    """Host-side prepared tables of the quantized scorers (no GPU needed)."""
    lib = _capi.load_library()
    d = ms.desc()
    dp = (ms.dimension + 15) // 16 * 16
    s = ctypes.c_float()
    isv = np.empty((ms.n_covariances, ms.dimension), dtype=np.float32)
    ln = np.empty(ms.n_covariances, dtype=np.float32)
    pm = np.empty((ms.n_entries, dp), dtype=np.uint8)
    cw = np.empty(ms.n_entries, dtype=np.int32)
    _capi.check(lib.gmm_prepare_quantized_host(ctypes.byref(d), _type_id(scorer_type), ctypes.byref(s),
                                               isv.ctypes.data_as(ctypes.c_void_p), ln.ctypes.data_as(ctypes.c_void_p),
                                               pm.ctypes.data_as(ctypes.c_void_p), cw.ctypes.data_as(ctypes.c_void_p)),
                "gmm_prepare_quantized_host")
    return {"scaling": s.value, "isv": isv, "log_norm": ln, "prepared_mean": pm, "constant_weight": cw}
