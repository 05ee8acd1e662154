"""In-memory mixture set (the data of Mm::MixtureSet, src/Mm/MixtureSet.hh:140-212)
and synthetic models of the shape SURVEY.md section 8(d) benchmarks on.

A MixtureSet holds numpy arrays; `desc()` returns the ctypes descriptor of
include/rasr_gmm.h (gmm_mixture_set) pointing into them (keep the MixtureSet
alive while the descriptor is used).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field

import numpy as np

from . import _capi


@dataclass
class MixtureSet:
    means: np.ndarray                # [n_means, D] f32
    variances: np.ndarray            # [n_covariances, D] f32 (Covariance::diagonal())
    density_mean: np.ndarray         # [n_densities] u32
    density_covariance: np.ndarray   # [n_densities] u32
    mixture_offsets: np.ndarray      # [n_mixtures + 1] u32
    mixture_densities: np.ndarray    # [n_entries] u32
    mixture_log_weights: np.ndarray  # [n_entries] f64 (Mm::Weight)
    _keep: list = field(default_factory=list, repr=False)

    def __post_init__(self):
        self.means = np.ascontiguousarray(self.means, dtype=np.float32)
        self.variances = np.ascontiguousarray(self.variances, dtype=np.float32)
        self.density_mean = np.ascontiguousarray(self.density_mean, dtype=np.uint32)
        self.density_covariance = np.ascontiguousarray(self.density_covariance, dtype=np.uint32)
        self.mixture_offsets = np.ascontiguousarray(self.mixture_offsets, dtype=np.uint32)
        self.mixture_densities = np.ascontiguousarray(self.mixture_densities, dtype=np.uint32)
        self.mixture_log_weights = np.ascontiguousarray(self.mixture_log_weights, dtype=np.float64)

    @property
    def dimension(self) -> int:
        return int(self.means.shape[1])

    @property
    def n_mixtures(self) -> int:
        return int(self.mixture_offsets.shape[0] - 1)

    @property
    def n_densities(self) -> int:
        return int(self.density_mean.shape[0])

    @property
    def n_entries(self) -> int:
        return int(self.mixture_offsets[-1])

    @property
    def n_covariances(self) -> int:
        return int(self.variances.shape[0])

    def desc(self) -> _capi.MixtureSetDesc:
        def p(a, t):
            return a.ctypes.data_as(ctypes.POINTER(t))
        d = _capi.MixtureSetDesc()
        d.dimension = self.dimension
        d.n_means = self.means.shape[0]
        d.means = p(self.means, ctypes.c_float)
        d.n_covariances = self.n_covariances
        d.variances = p(self.variances, ctypes.c_float)
        d.n_densities = self.n_densities
        d.density_mean = p(self.density_mean, ctypes.c_uint32)
        d.density_covariance = p(self.density_covariance, ctypes.c_uint32)
        d.n_mixtures = self.n_mixtures
        d.mixture_offsets = p(self.mixture_offsets, ctypes.c_uint32)
        d.mixture_densities = p(self.mixture_densities, ctypes.c_uint32)
        d.mixture_log_weights = p(self.mixture_log_weights, ctypes.c_double)
        return d

    def save_npz(self, path: str) -> None:
        np.savez_compressed(path, means=self.means, variances=self.variances, density_mean=self.density_mean,
                            density_covariance=self.density_covariance, mixture_offsets=self.mixture_offsets,
                            mixture_densities=self.mixture_densities, mixture_log_weights=self.mixture_log_weights)

    @staticmethod
    def load_npz(path: str) -> "MixtureSet":
        z = np.load(path, allow_pickle=False)
        return MixtureSet(z["means"], z["variances"], z["density_mean"], z["density_covariance"],
                          z["mixture_offsets"], z["mixture_densities"], z["mixture_log_weights"])


def _from_desc(d: _capi.MixtureSetDesc) -> MixtureSet:
    def arr(ptr, n, dtype):
        if n == 0:
            return np.zeros(0, dtype=dtype)
        return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True)
    D = int(d.dimension)
    n_entries = int(d.mixture_offsets[d.n_mixtures]) if d.mixture_offsets else 0
    return MixtureSet(
        means=arr(d.means, d.n_means * D, np.float32).reshape(d.n_means, D),
        variances=arr(d.variances, d.n_covariances * D, np.float32).reshape(d.n_covariances, D),
        density_mean=arr(d.density_mean, d.n_densities, np.uint32),
        density_covariance=arr(d.density_covariance, d.n_densities, np.uint32),
        mixture_offsets=arr(d.mixture_offsets, d.n_mixtures + 1, np.uint32),
        mixture_densities=arr(d.mixture_densities, n_entries, np.uint32),
        mixture_log_weights=arr(d.mixture_log_weights, n_entries, np.float64))


def estimator_config(**kw) -> _capi.EstimatorConfig:
    """gmm_estimator_config with the reference defaults, overridden by keyword (minimum_observation_weight,
    minimum_relative_weight, minimum_variance, allow_zero_weights, normalize_mixture_weights)."""
    cfg = _capi.EstimatorConfig()
    _capi.load_library().gmm_default_estimator_config(ctypes.byref(cfg))
    for k, v in kw.items():
        if not hasattr(cfg, k):
            raise TypeError(f"unknown estimator parameter {k}")
        setattr(cfg, k, v)
    return cfg


def read_mixture_set(path: str, dimension_offset: int = 0, reduced_dimension: int = 0, **estimator) -> MixtureSet:
    """Read a RASR mixture set through the C-ABI (gmm_mixture_set_read_config, include/rasr_gmm_io.h;
    Mm::Module_::readMixtureSet, src/Mm/Module.cc:152-182, with the reduced-mixture-set-dimension[-offset]
    parameters): ".pms" / ".gz" names as text, any other name as a binary maximum-likelihood estimator file,
    estimated with the given parameters (estimator_config)."""
    lib = _capi.load_library()
    d = _capi.MixtureSetDesc()
    cfg = estimator_config(**estimator)
    _capi.check(lib.gmm_mixture_set_read_config(os.fsencode(path), ctypes.byref(cfg), dimension_offset,
                                                reduced_dimension, ctypes.byref(d)), "gmm_mixture_set_read")
    try:
        return _from_desc(d)
    finally:
        lib.gmm_mixture_set_free(ctypes.byref(d))


def parse_mixture_set(data: bytes, dimension_offset: int = 0, reduced_dimension: int = 0) -> MixtureSet:
    """gmm_mixture_set_parse: the same reader over in-memory (plain or gzip) bytes."""
    lib = _capi.load_library()
    d = _capi.MixtureSetDesc()
    buf = ctypes.create_string_buffer(data, len(data))
    _capi.check(lib.gmm_mixture_set_parse(buf, len(data), dimension_offset, reduced_dimension, ctypes.byref(d)),
                "gmm_mixture_set_parse")
    try:
        return _from_desc(d)
    finally:
        lib.gmm_mixture_set_free(ctypes.byref(d))


def estimate_mixture_set(data: bytes, **estimator) -> MixtureSet:
    """gmm_mixture_set_estimate: the mixture set a binary estimator file's bytes describe."""
    lib = _capi.load_library()
    d = _capi.MixtureSetDesc()
    cfg = estimator_config(**estimator)
    buf = ctypes.create_string_buffer(data, len(data))
    _capi.check(lib.gmm_mixture_set_estimate(buf, len(data), ctypes.byref(cfg), ctypes.byref(d)),
                "gmm_mixture_set_estimate")
    try:
        return _from_desc(d)
    finally:
        lib.gmm_mixture_set_free(ctypes.byref(d))


def write_mixture_set(path: str, ms: MixtureSet, precision: int = 6) -> None:
    """gmm_mixture_set_write: MixtureSet::write text (src/Mm/MixtureSet.cc:142-168), gzip for *.gz."""
    lib = _capi.load_library()
    d = ms.desc()
    _capi.check(lib.gmm_mixture_set_write(os.fsencode(path), ctypes.byref(d), precision), "gmm_mixture_set_write")


def synthetic_mixture_set(n_mixtures: int, densities_per_mixture, dimension: int, seed: int = 1234,
                          n_covariances: int = 1, weights: str = "uniform", tying: str | None = None) -> MixtureSet:
    """SURVEY.md section 8(d) synthetic model.

    pooled variance  s2_k = 0.5 + |N(0,1)|;  means ~ N(0,1);  one mean per density;
    weights: "uniform" -> log(1/K_m);  "random" -> normalized Dirichlet(1) draws.
    densities_per_mixture: int, or a sequence of per-mixture counts (ragged models).
    n_covariances > 1 assigns every density a random covariance (untied variant).
    tying (RASR's covariance-tying, src/Mm/Module.cc:54-58, 127-136) overrides n_covariances:
    "pooled" one covariance, "mixture-specific" one per mixture, "none" one per density.
    """
    if tying is not None:
        if tying not in ("pooled", "mixture-specific", "none"):
            raise ValueError(tying)
        counts = (np.full(n_mixtures, int(densities_per_mixture), dtype=np.int64) if np.isscalar(densities_per_mixture)
                  else np.asarray(densities_per_mixture, dtype=np.int64))
        base = synthetic_mixture_set(n_mixtures, counts, dimension, seed, 1, weights)
        if tying == "pooled":
            return base
        n = int(counts.sum())
        c = n_mixtures if tying == "mixture-specific" else n
        rng = np.random.Generator(np.random.PCG64(seed + 7))
        var = (0.5 + np.abs(rng.standard_normal((max(c, 1), dimension), dtype=np.float32))).astype(np.float32)
        dcov = (np.repeat(np.arange(n_mixtures, dtype=np.uint32), counts) if tying == "mixture-specific"
                else np.arange(n, dtype=np.uint32))
        return MixtureSet(means=base.means, variances=var, density_mean=base.density_mean, density_covariance=dcov,
                          mixture_offsets=base.mixture_offsets, mixture_densities=base.mixture_densities,
                          mixture_log_weights=base.mixture_log_weights)
    rng = np.random.Generator(np.random.PCG64(seed))
    if np.isscalar(densities_per_mixture):
        counts = np.full(n_mixtures, int(densities_per_mixture), dtype=np.int64)
    else:
        counts = np.asarray(densities_per_mixture, dtype=np.int64)
        assert counts.shape[0] == n_mixtures
    n = int(counts.sum())
    variances = (0.5 + np.abs(rng.standard_normal((n_covariances, dimension), dtype=np.float32))).astype(np.float32)
    means = rng.standard_normal((n, dimension), dtype=np.float32)
    offsets = np.zeros(n_mixtures + 1, dtype=np.uint32)
    offsets[1:] = np.cumsum(counts)
    if n_covariances == 1:
        dcov = np.zeros(n, dtype=np.uint32)
    else:
        dcov = rng.integers(0, n_covariances, size=n, dtype=np.uint32)
    if weights == "uniform":
        logw = np.concatenate([np.full(c, np.log(1.0 / c)) for c in counts]) if n else np.zeros(0)
    elif weights == "random":
        parts = []
        for c in counts:
            w = rng.exponential(1.0, size=int(c))
            parts.append(np.log(w / w.sum()))
        logw = np.concatenate(parts) if parts else np.zeros(0)
    else:
        raise ValueError(weights)
    return MixtureSet(means=means, variances=variances, density_mean=np.arange(n, dtype=np.uint32),
                      density_covariance=dcov, mixture_offsets=offsets,
                      mixture_densities=np.arange(n, dtype=np.uint32), mixture_log_weights=logw)


def synthetic_frames(n_frames: int, dimension: int, seed: int = 4321) -> np.ndarray:
    """Feature vectors x ~ N(0,1), [n_frames, D] f32."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.standard_normal((n_frames, dimension), dtype=np.float32)


def ragged_counts(n_mixtures: int, total: int, low: int = 64, high: int = 256, seed: int = 99) -> np.ndarray:
    """K_m ~ U[low, high] rescaled so that sum K_m == total (SURVEY.md 8(d) ragged variant)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    k = rng.integers(low, high + 1, size=n_mixtures).astype(np.float64)
    k = np.maximum(1, np.round(k * total / k.sum())).astype(np.int64)
    diff = total - int(k.sum())
    i = 0
    while diff != 0:
        step = 1 if diff > 0 else -1
        if k[i % n_mixtures] + step >= 1:
            k[i % n_mixtures] += step
            diff -= step
        i += 1
    return k
