"""TEST INFRASTRUCTURE ONLY -- ctypes binding of oracle/_build/libgmm_oracle.so.

CPU restatement of RASR's feature scorers (parity checker + CPU baseline).
Parity status: UNPINNED (gmm_oracle.h explains why).  Works on any object with
the MixtureSet attributes (means, variances, density_mean, density_covariance,
mixture_offsets, mixture_densities, mixture_log_weights).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "_build", "libgmm_oracle.so")

_u32p = ctypes.POINTER(ctypes.c_uint32)
_f32p = ctypes.POINTER(ctypes.c_float)
_f64p = ctypes.POINTER(ctypes.c_double)
_vp = ctypes.c_void_p


class OrcMixtureSet(ctypes.Structure):
    _fields_ = [("dimension", ctypes.c_uint32), ("n_means", ctypes.c_uint32), ("means", _f32p),
                ("n_covariances", ctypes.c_uint32), ("variances", _f32p), ("n_densities", ctypes.c_uint32),
                ("density_mean", _u32p), ("density_covariance", _u32p), ("n_mixtures", ctypes.c_uint32),
                ("mixture_offsets", _u32p), ("mixture_densities", _u32p), ("mixture_log_weights", _f64p)]


class OrcSimdModel(ctypes.Structure):
    _fields_ = [("dimension", ctypes.c_uint32), ("padded_dimension", ctypes.c_uint32),
                ("n_covariances", ctypes.c_uint32), ("n_entries", ctypes.c_uint32), ("scaling", ctypes.c_float),
                ("scaling_squared", ctypes.c_float), ("inverse_quantization_factor", ctypes.c_float),
                ("isv", _f32p), ("log_norm", _f32p), ("prepared_mean", ctypes.POINTER(ctypes.c_uint8)),
                ("constant_weight", ctypes.POINTER(ctypes.c_int32)), ("entry_covariance", _u32p)]


class OrcFloatModel(ctypes.Structure):
    _fields_ = [("dimension", ctypes.c_uint32), ("n_covariances", ctypes.c_uint32), ("n_entries", ctypes.c_uint32),
                ("isv", _f32p), ("log_norm", _f32p), ("minus2_log_weight", _f32p)]


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    lib = ctypes.CDLL(LIB)
    sig = {
        "orc_inverse_sqrt": (ctypes.c_float, [ctypes.c_float]),
        "orc_quantize": (ctypes.c_uint8, [ctypes.c_float]),
        "orc_gauss_log_norm": (ctypes.c_double, [_f32p, ctypes.c_uint32]),
        "orc_quantization_scaling_factor": (ctypes.c_float, [ctypes.c_float, ctypes.c_float]),
        "orc_constant_weight": (ctypes.c_int32, [ctypes.c_float, ctypes.c_double, ctypes.c_float]),
        "orc_simd_final_score": (ctypes.c_float, [ctypes.c_int32, ctypes.c_float]),
        "orc_batch_int_constant": (ctypes.c_int32, [ctypes.c_float, ctypes.c_float, ctypes.c_double]),
        "orc_batch_int_final_score": (ctypes.c_float, [ctypes.c_int32, ctypes.c_float]),
        "orc_float_distance": (ctypes.c_float, [_f32p, _f32p, _f32p, ctypes.c_uint32]),
        "orc_quantize_array": (None, [_vp, ctypes.c_uint32, _vp]),
        "orc_batch_int_prepare": (ctypes.c_int, [ctypes.POINTER(OrcMixtureSet), _f32p, _vp, _vp]),
        "orc_simd_prepare": (ctypes.c_int, [ctypes.POINTER(OrcMixtureSet), ctypes.POINTER(OrcSimdModel)]),
        "orc_simd_free": (None, [ctypes.POINTER(OrcSimdModel)]),
        "orc_simd_quantize_frame": (None, [ctypes.POINTER(OrcSimdModel), _f32p, _vp]),
        "orc_simd_score": (ctypes.c_int, [ctypes.POINTER(OrcSimdModel), ctypes.POINTER(OrcMixtureSet), _vp,
                                          ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, _vp, ctypes.c_int]),
        "orc_float_prepare": (ctypes.c_int, [ctypes.POINTER(OrcMixtureSet), ctypes.c_float, ctypes.c_float,
                                             ctypes.POINTER(OrcFloatModel)]),
        "orc_float_free": (None, [ctypes.POINTER(OrcFloatModel)]),
        "orc_float_score": (ctypes.c_int, [ctypes.POINTER(OrcFloatModel), ctypes.POINTER(OrcMixtureSet), _vp,
                                           ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, ctypes.c_int]),
        "orc_float_sum_score": (ctypes.c_int, [ctypes.POINTER(OrcFloatModel), ctypes.POINTER(OrcMixtureSet), _vp,
                                               ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, ctypes.c_int]),
        "orc_batch_int_score": (ctypes.c_int, [ctypes.POINTER(OrcMixtureSet), _vp, ctypes.c_uint32,
                                               ctypes.c_uint32, _vp, ctypes.c_int]),
        "orc_batch_float_score": (ctypes.c_int, [ctypes.POINTER(OrcMixtureSet), _vp, ctypes.c_uint32,
                                                 ctypes.c_uint32, _vp, ctypes.c_int]),
        "orc_batch_int_score_sel": (ctypes.c_int, [ctypes.POINTER(OrcMixtureSet), _vp, ctypes.c_uint32,
                                                   ctypes.c_uint32, _vp, ctypes.c_int, _vp, _vp, ctypes.c_uint32]),
        "orc_batch_float_score_sel": (ctypes.c_int, [ctypes.POINTER(OrcMixtureSet), _vp, ctypes.c_uint32,
                                                     ctypes.c_uint32, _vp, ctypes.c_int, _vp, _vp, ctypes.c_uint32,
                                                     ctypes.c_float]),
        "orc_batch_float_tables": (ctypes.c_int, [ctypes.POINTER(OrcMixtureSet), _vp, _vp, _vp]),
        "orc_batch_int_tables": (ctypes.c_int, [ctypes.POINTER(OrcMixtureSet), _vp, _vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


class _Desc:
    """Keeps contiguous copies alive and exposes the C descriptor."""

    def __init__(self, ms):
        self.means = np.ascontiguousarray(ms.means, dtype=np.float32)
        self.variances = np.ascontiguousarray(ms.variances, dtype=np.float32)
        self.dm = np.ascontiguousarray(ms.density_mean, dtype=np.uint32)
        self.dc = np.ascontiguousarray(ms.density_covariance, dtype=np.uint32)
        self.mo = np.ascontiguousarray(ms.mixture_offsets, dtype=np.uint32)
        self.md = np.ascontiguousarray(ms.mixture_densities, dtype=np.uint32)
        self.lw = np.ascontiguousarray(ms.mixture_log_weights, dtype=np.float64)
        d = OrcMixtureSet()
        d.dimension = self.means.shape[1]
        d.n_means = self.means.shape[0]
        d.means = self.means.ctypes.data_as(_f32p)
        d.n_covariances = self.variances.shape[0]
        d.variances = self.variances.ctypes.data_as(_f32p)
        d.n_densities = self.dm.shape[0]
        d.density_mean = self.dm.ctypes.data_as(_u32p)
        d.density_covariance = self.dc.ctypes.data_as(_u32p)
        d.n_mixtures = self.mo.shape[0] - 1
        d.mixture_offsets = self.mo.ctypes.data_as(_u32p)
        d.mixture_densities = self.md.ctypes.data_as(_u32p)
        d.mixture_log_weights = self.lw.ctypes.data_as(_f64p)
        self.c = d
        self.n_mixtures = int(d.n_mixtures)
        self.n_entries = int(self.mo[-1])


def _frames(frames):
    f = np.ascontiguousarray(frames, dtype=np.float32)
    return f, f.shape[0], f.shape[1]


class OracleSimd:
    """SIMD-diagonal-maximum restated (SimdFeatureScorer.cc)."""

    def __init__(self, ms):
        self.lib = load()
        self.d = _Desc(ms)
        self.m = OrcSimdModel()
        rc = self.lib.orc_simd_prepare(ctypes.byref(self.d.c), ctypes.byref(self.m))
        if rc != 0:
            raise ValueError("orc_simd_prepare failed")
        D, Dp, C, E = self.m.dimension, self.m.padded_dimension, self.m.n_covariances, self.m.n_entries
        self.scaling = self.m.scaling
        self.scaling_squared = self.m.scaling_squared
        self.inverse_quantization_factor = self.m.inverse_quantization_factor
        self.isv = np.ctypeslib.as_array(self.m.isv, shape=(C * D,)).reshape(C, D).copy()
        self.log_norm = np.ctypeslib.as_array(self.m.log_norm, shape=(C,)).copy()
        self.prepared_mean = (np.ctypeslib.as_array(self.m.prepared_mean, shape=(E * Dp,)).reshape(E, Dp).copy()
                              if E else np.zeros((0, Dp), np.uint8))
        self.constant_weight = (np.ctypeslib.as_array(self.m.constant_weight, shape=(E,)).copy()
                                if E else np.zeros(0, np.int32))

    def __del__(self):
        try:
            self.lib.orc_simd_free(ctypes.byref(self.m))
        except Exception:
            pass

    def quantize_frame(self, x):
        x = np.ascontiguousarray(x, dtype=np.float32)
        out = np.empty((self.m.n_covariances, self.m.padded_dimension), dtype=np.uint8)
        self.lib.orc_simd_quantize_frame(ctypes.byref(self.m), x.ctypes.data_as(_f32p),
                                         out.ctypes.data_as(ctypes.c_void_p))
        return out

    def score(self, frames, n_threads: int = 1):
        f, n, stride = _frames(frames)
        M = self.d.n_mixtures
        scores = np.empty((M, n), np.float32)
        best = np.empty((M, n), np.uint32)
        raw = np.empty((M, n), np.int32)
        self.lib.orc_simd_score(ctypes.byref(self.m), ctypes.byref(self.d.c), f.ctypes.data_as(_vp), n, stride,
                                scores.ctypes.data_as(_vp), best.ctypes.data_as(_vp), raw.ctypes.data_as(_vp),
                                int(n_threads))
        return scores, best, raw


class OracleFloat:
    """diagonal-maximum restated (GaussDiagonalMaximumFeatureScorer.cc)."""

    def __init__(self, ms, mixture_weight_scale: float = 1.0, gaussian_scale: float = 1.0):
        self.lib = load()
        self.d = _Desc(ms)
        self.m = OrcFloatModel()
        rc = self.lib.orc_float_prepare(ctypes.byref(self.d.c), mixture_weight_scale, gaussian_scale,
                                        ctypes.byref(self.m))
        if rc != 0:
            raise ValueError("orc_float_prepare failed")

    def __del__(self):
        try:
            self.lib.orc_float_free(ctypes.byref(self.m))
        except Exception:
            pass

    _score_fn = "orc_float_score"

    def score(self, frames, n_threads: int = 1):
        f, n, stride = _frames(frames)
        M = self.d.n_mixtures
        scores = np.empty((M, n), np.float32)
        best = np.empty((M, n), np.uint32)
        getattr(self.lib, self._score_fn)(ctypes.byref(self.m), ctypes.byref(self.d.c), f.ctypes.data_as(_vp), n,
                                          stride, scores.ctypes.data_as(_vp), best.ctypes.data_as(_vp),
                                          int(n_threads))
        return scores, best


class OracleFloatSum(OracleFloat):
    """diagonal-sum restated (GaussDiagonalSumFeatureScorer, GaussDiagonalMaximumFeatureScorer.cc:221-298):
    -log sum_d exp(-s_d) with f32 density scores, best density as diagonal-maximum."""

    _score_fn = "orc_float_sum_score"


def batch_int_score(ms, frames, n_threads: int = 1):
    lib = load()
    d = _Desc(ms)
    f, n, stride = _frames(frames)
    scores = np.empty((d.n_mixtures, n), np.float32)
    if lib.orc_batch_int_score(ctypes.byref(d.c), f.ctypes.data_as(_vp), n, stride, scores.ctypes.data_as(_vp),
                               int(n_threads)) != 0:
        raise ValueError("orc_batch_int_score failed")
    return scores


def batch_float_score(ms, frames, n_threads: int = 1):
    lib = load()
    d = _Desc(ms)
    f, n, stride = _frames(frames)
    scores = np.empty((d.n_mixtures, n), np.float32)
    if lib.orc_batch_float_score(ctypes.byref(d.c), f.ctypes.data_as(_vp), n, stride, scores.ctypes.data_as(_vp),
                                 int(n_threads)) != 0:
        raise ValueError("orc_batch_float_score failed")
    return scores


def batch_fast_score(ms, frames):
    """batch-diagonal-maximum-fast restated: BatchUnrolledIntFeatureScorer::fillScoreCache
    (src/Mm/BatchFeatureScorer.cc:558-604) over BatchIntFeatureScorer::init's tables (cc:339-380).  The
    unrolled loop always loads 3 x 16 feature bytes and 3 x 16 mean bytes and advances the mean pointer by
    the fixed 48 bytes (`mean += Dimension`, cc:591), while init lays the means out at paddedDimension_
    (cc:367-375).  For a padded dimension of 48 (dimension 33..48) that is batch-int's arithmetic; for 16
    or 32 the loads run into the next buffered features and the next densities' means, and the last
    mixture's past the end of the allocation (cc:362-363), so the reference result is undefined there and
    this restatement refuses, as the GPU scorer does."""
    d = _Desc(ms)
    D = ms.means.shape[1]
    dp = (D + 15) // 16 * 16
    if dp != 48:
        raise ValueError(f"padded dimension {dp}: the reference's unrolled loads leave its own rows")
    scale, _, const = batch_int_prepare(ms)
    var = np.empty(dp, np.float32)
    means = np.empty((d.n_entries, dp), np.uint8)
    if load().orc_batch_int_tables(ctypes.byref(d.c), var.ctypes.data_as(_vp), means.ctypes.data_as(_vp)) != 0:
        raise ValueError("orc_batch_int_tables failed")
    f, n, _ = _frames(frames)
    feats = np.zeros((n, dp), np.uint8)
    feats[:, :D] = quantize_array(f * var[:D]).reshape(n, D)  # setFeature: q(f * variance_) (cc:382-388)
    off = d.mo.astype(np.int64)
    scores = np.empty((d.n_mixtures, n), np.float32)
    for m in range(d.n_mixtures):
        mm = means[off[m]:off[m + 1]].reshape(-1, 48).astype(np.int32)  # the 48-byte stride of cc:591
        best = np.full(n, 2147483647, np.int64)
        if mm.shape[0]:
            dist = ((feats[:, None, :].astype(np.int32) - mm[None]) ** 2).sum(-1)  # addDistance x 3 blocks
            tmp = dist + const[off[m]:off[m + 1]][None].astype(np.int64)
            best = np.minimum(best, tmp.min(1))  # strict < from INT_MAX (cc:593-597)
        scores[m] = best.astype(np.int32).astype(np.float32) / np.float32(scale)  # (f32)best / scale_ (cc:602)
    return scores


def inverse_sqrt(x: float) -> float:
    return load().orc_inverse_sqrt(x)


def quantize(x: float) -> int:
    return load().orc_quantize(x)


def gauss_log_norm(v) -> float:
    v = np.ascontiguousarray(v, dtype=np.float32)
    return load().orc_gauss_log_norm(v.ctypes.data_as(_f32p), v.shape[0])


def quantization_scaling_factor(a: float, b: float) -> float:
    return load().orc_quantization_scaling_factor(a, b)


def constant_weight(s2: float, logw: float, lognorm: float) -> int:
    return load().orc_constant_weight(s2, logw, lognorm)


def simd_final_score(q: int, s2: float) -> float:
    return load().orc_simd_final_score(q, s2)


def float_distance(feature, mean, isv) -> float:
    f = np.ascontiguousarray(feature, np.float32)
    m = np.ascontiguousarray(mean, np.float32)
    i = np.ascontiguousarray(isv, np.float32)
    return load().orc_float_distance(f.ctypes.data_as(_f32p), m.ctypes.data_as(_f32p), i.ctypes.data_as(_f32p),
                                     f.shape[0])


def quantize_array(x) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32).ravel()
    out = np.empty(x.shape[0], dtype=np.uint8)
    load().orc_quantize_array(x.ctypes.data_as(_vp), x.shape[0], out.ctypes.data_as(_vp))
    return out


def batch_int_prepare(ms):
    """(scale_, variance_ [D], constants_ [entries]) of BatchIntFeatureScorer::init."""
    d = _Desc(ms)
    scale = ctypes.c_float()
    var = np.empty(ms.means.shape[1], np.float32)
    const = np.empty(d.n_entries, np.int32)
    if load().orc_batch_int_prepare(ctypes.byref(d.c), ctypes.byref(scale), var.ctypes.data_as(_vp),
                                    const.ctypes.data_as(_vp)) != 0:
        raise ValueError("orc_batch_int_prepare failed")
    return scale.value, var, const


# ---------------------------------------------------------------------------
# preselection-batch-float / -int (oracle/presel_oracle.cc + the batch scorers with a selector)
# ---------------------------------------------------------------------------
PRESEL_LIB = os.path.join(_HERE, "_build", "libpresel_oracle.so")
_presel = None


def load_presel() -> ctypes.CDLL:
    global _presel
    if _presel is not None:
        return _presel
    if not os.path.exists(PRESEL_LIB):
        build()
    lib = ctypes.CDLL(PRESEL_LIB)
    u32 = ctypes.c_uint32
    for name, args in {
        "orc_libc_rand_sequence": [u32, u32, _vp],
        "orc_cluster_build_f32": [_vp, u32, u32, u32, u32, _vp, _vp],
        "orc_cluster_build_u8": [_vp, u32, u32, u32, u32, _vp, _vp],
        "orc_select_clusters_f32": [_vp, u32, _vp, u32, u32, u32, _vp],
        "orc_select_clusters_u8": [_vp, u32, _vp, u32, u32, u32, _vp],
    }.items():
        f = getattr(lib, name)
        f.restype = ctypes.c_int
        f.argtypes = args
    _presel = lib
    return lib


def libc_rand_sequence(seed: int, n: int) -> np.ndarray:
    out = np.empty(n, np.int32)
    load_presel().orc_libc_rand_sequence(seed, n, out.ctypes.data_as(_vp))
    return out


class OraclePresel:
    """preselection-batch-float (kind "float") / preselection-batch-int (kind "int") restated:
    DensityClustering over the batch scorer's prepared means, per-frame selection of the n_select
    nearest clusters, the batch scorer over the selected densities (backoff score for a float
    mixture without any, BatchFeatureScorer.cc:282-288)."""

    def __init__(self, ms, kind: str, clusters: int = 256, select: int = 32, iterations: int = 5,
                 backoff: float = 40000.0):
        assert kind in ("float", "int")
        self.kind = kind
        self.ms = ms
        self._d = _Desc(ms)
        lib = load()
        D = int(self._d.c.dimension)
        E = self._d.n_entries
        if kind == "float":
            self.dp = (D + 7) // 8 * 8
            self.variance = np.zeros(self.dp, np.float32)
            self.means = np.zeros((E, self.dp), np.float32)
            consts = np.zeros(E, np.float32)
            rc = lib.orc_batch_float_tables(ctypes.byref(self._d.c), self.variance.ctypes.data_as(_vp),
                                            self.means.ctypes.data_as(_vp), consts.ctypes.data_as(_vp))
        else:
            self.dp = (D + 15) // 16 * 16
            self.variance = np.zeros(self.dp, np.float32)
            self.means = np.zeros((E, self.dp), np.uint8)
            rc = lib.orc_batch_int_tables(ctypes.byref(self._d.c), self.variance.ctypes.data_as(_vp),
                                          self.means.ctypes.data_as(_vp))
        if rc != 0:
            raise ValueError("batch tables failed")
        # DensityClusteringBase::init (DensityClustering.cc:48-61)
        self.n_clusters = min(int(clusters), E)
        self.n_select = int(select)
        if self.n_select > self.n_clusters:
            raise ValueError("select-clusters exceeds the number of clusters")
        self.backoff = float(backoff)
        self.cluster_of_entry = np.zeros(E, np.uint8)
        self.cluster_means = np.zeros((self.n_clusters, self.dp), self.means.dtype)
        fn = load_presel().orc_cluster_build_f32 if kind == "float" else load_presel().orc_cluster_build_u8
        if fn(self.means.ctypes.data_as(_vp), E, self.dp, self.n_clusters, int(iterations),
              self.cluster_of_entry.ctypes.data_as(_vp), self.cluster_means.ctypes.data_as(_vp)) != 0:
            raise ValueError("cluster build failed")

    def features(self, frames):
        """setFeature (BatchFeatureScorer.cc:137-142 / 382-388): [n][Dp]"""
        f, n, _ = _frames(frames)
        D = int(self._d.c.dimension)
        x = f[:, :D] * self.variance[None, :D]
        if self.kind == "float":
            out = np.zeros((n, self.dp), np.float32)
            out[:, :D] = x
            return out
        out = np.zeros((n, self.dp), np.uint8)
        out[:, :D] = quantize_array(x).reshape(n, D)
        return out

    def select(self, frames) -> np.ndarray:
        """activeClusters_ per frame: [n][n_clusters] 0/1 (DensityClustering.tcc:151-176)"""
        feats = np.ascontiguousarray(self.features(frames))
        n = feats.shape[0]
        sel = np.zeros((n, self.n_clusters), np.uint8)
        fn = load_presel().orc_select_clusters_f32 if self.kind == "float" else load_presel().orc_select_clusters_u8
        fn(feats.ctypes.data_as(_vp), n, self.cluster_means.ctypes.data_as(_vp), self.n_clusters, self.dp,
           self.n_select, sel.ctypes.data_as(_vp))
        return sel

    def score(self, frames, n_threads: int = 1, selection=None):
        f, n, stride = _frames(frames)
        sel = np.ascontiguousarray(self.select(f) if selection is None else selection, dtype=np.uint8)
        scores = np.empty((self._d.n_mixtures, n), np.float32)
        lib = load()
        if self.kind == "float":
            rc = lib.orc_batch_float_score_sel(ctypes.byref(self._d.c), f.ctypes.data_as(_vp), n, stride,
                                               scores.ctypes.data_as(_vp), int(n_threads),
                                               self.cluster_of_entry.ctypes.data_as(_vp), sel.ctypes.data_as(_vp),
                                               self.n_clusters, self.backoff)
        else:
            rc = lib.orc_batch_int_score_sel(ctypes.byref(self._d.c), f.ctypes.data_as(_vp), n, stride,
                                             scores.ctypes.data_as(_vp), int(n_threads),
                                             self.cluster_of_entry.ctypes.data_as(_vp), sel.ctypes.data_as(_vp),
                                             self.n_clusters)
        if rc != 0:
            raise ValueError("preselection score failed")
        return scores
