"""ctypes binding of the C-ABI in include/rasr_gmm.h (librasr_gmm.so).

The library is the product: there is no Python or CPU fallback.  If the shared
object is missing, loading raises immediately (build it with `make` or
`python -c "import __graft_entry__ as g; g.build()"`).
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# RASR_GMM_LIB selects another build of the same library (kernel A/B variants, scripts/ab_bench.py)
LIB_PATH = os.environ.get("RASR_GMM_LIB") or os.path.join(_HERE, "lib", "librasr_gmm.so")

GMM_OK = 0
GMM_FLAG_NATIVE_F32 = 1  # gmm_scorer_config.flags
GMM_FLAG_SPLIT_TILE16 = 2
GMM_FLAG_SPLIT_TILE32 = 4
GMM_FLAG_REFERENCE_ORDER = 8  # diagonal-maximum / batch-float in the reference's f32 operation order
GMM_FLAG_FULL_KEYS = 16  # batch-int / -fast: (score, density) keys instead of the score-only class layout
GMM_FLAG_NO_SCORE_ONLY_TWIN = 32  # SIMD: no score-only copy of the model (callers that always want best densities)
GMM_FLAG_CACHE_ARCHIVE_READ_ONLY = 64  # preselection: read the cached clustering, never write it
GMM_CLUSTERING = {0: "built", 1: "written", 2: "cached"}  # gmm_scorer_clustering_source

# Mm::Module_::FeatureScorerType values (src/Mm/Module.hh:48-70)
BATCH_DIAGONAL_MAXIMUM_FLOAT = 0
BATCH_PRESELECTION_FLOAT = 1
BATCH_PRESELECTION_INT = 2
BATCH_DIAGONAL_MAXIMUM_INT = 3
BATCH_DIAGONAL_MAXIMUM_FAST = 4
DIAGONAL_MAXIMUM = 5
SIMD_DIAGONAL_MAXIMUM = 9
DIAGONAL_SUM = 12  # diagonalSum (no registration string in the reference factory)

SCORER_TYPES = {
    "batch-diagonal-maximum-float": BATCH_DIAGONAL_MAXIMUM_FLOAT,
    "batch-diagonal-maximum-int": BATCH_DIAGONAL_MAXIMUM_INT,
    "batch-diagonal-maximum-fast": BATCH_DIAGONAL_MAXIMUM_FAST,
    "preselection-batch-float": BATCH_PRESELECTION_FLOAT,
    "preselection-batch-int": BATCH_PRESELECTION_INT,
    "diagonal-maximum": DIAGONAL_MAXIMUM,
    "SIMD-diagonal-maximum": SIMD_DIAGONAL_MAXIMUM,
    "diagonal-sum": DIAGONAL_SUM,
}

_u32p = ctypes.POINTER(ctypes.c_uint32)
_f32p = ctypes.POINTER(ctypes.c_float)
_f64p = ctypes.POINTER(ctypes.c_double)


class MixtureSetDesc(ctypes.Structure):
    _fields_ = [
        ("dimension", ctypes.c_uint32),
        ("n_means", ctypes.c_uint32),
        ("means", _f32p),
        ("n_covariances", ctypes.c_uint32),
        ("variances", _f32p),
        ("n_densities", ctypes.c_uint32),
        ("density_mean", _u32p),
        ("density_covariance", _u32p),
        ("n_mixtures", ctypes.c_uint32),
        ("mixture_offsets", _u32p),
        ("mixture_densities", _u32p),
        ("mixture_log_weights", _f64p),
    ]


class ScorerConfig(ctypes.Structure):
    _fields_ = [
        ("mixture_weight_scale", ctypes.c_float),
        ("gaussian_scale", ctypes.c_float),
        ("score_scale", ctypes.c_float),
        ("max_frames", ctypes.c_uint32),
        ("mixture_begin", ctypes.c_uint32),
        ("mixture_end", ctypes.c_uint32),
        ("flags", ctypes.c_uint32),
        ("clusters", ctypes.c_uint32),
        ("select_clusters", ctypes.c_uint32),
        ("clustering_iterations", ctypes.c_uint32),
        ("backoff_score", ctypes.c_float),
        ("cache_archive", ctypes.c_char_p),
    ]


class EstimatorConfig(ctypes.Structure):
    _fields_ = [
        ("minimum_observation_weight", ctypes.c_double),
        ("minimum_relative_weight", ctypes.c_double),
        ("minimum_variance", ctypes.c_double),
        ("allow_zero_weights", ctypes.c_uint32),
        ("normalize_mixture_weights", ctypes.c_uint32),
    ]


GMM_HOST_KEEP_BEST = 1
GMM_HOST_FRAME_MAJOR = 2
GMM_HOST_LAZY_BEST = 4
GMM_HOST_ASYNC = 8
# gmm_scorer_create_sharded: the per-frame reduce of mixtures split between GPUs
GMM_EXCHANGE = {"auto": 0, "rccl": 1, "copy": 2}

# (name, restype, argtypes) for every function declared in include/rasr_gmm.h and rasr_gmm_io.h
PROTOTYPES = [
    ("gmm_default_config", None, [ctypes.POINTER(ScorerConfig)]),
    ("gmm_scorer_create", ctypes.c_int,
     [ctypes.POINTER(MixtureSetDesc), ctypes.c_int, ctypes.POINTER(ScorerConfig), ctypes.c_int,
      ctypes.POINTER(ctypes.c_void_p)]),
    ("gmm_scorer_destroy", ctypes.c_int, [ctypes.c_void_p]),
    ("gmm_scorer_n_mixtures", ctypes.c_uint32, [ctypes.c_void_p]),
    ("gmm_scorer_dimension", ctypes.c_uint32, [ctypes.c_void_p]),
    ("gmm_scorer_n_covariances", ctypes.c_uint32, [ctypes.c_void_p]),
    ("gmm_scorer_type_of", ctypes.c_int, [ctypes.c_void_p]),
    ("gmm_score_device", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
      ctypes.c_uint32, ctypes.c_void_p]),
    ("gmm_score_host", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
      ctypes.c_uint32]),
    ("gmm_score_host_ring", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)]),
    ("gmm_host_call_wait", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
    ("gmm_fetch_best_density", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32]),
    ("gmm_best_density_pairs", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]),
    ("gmm_best_density_pairs_device", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
      ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    ("gmm_host_alloc", ctypes.c_int, [ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]),
    ("gmm_host_free", ctypes.c_int, [ctypes.c_void_p]),
    ("gmm_scorer_quantization", ctypes.c_int, [ctypes.c_void_p, _f32p, _f32p]),
    ("gmm_scorer_multiply_and_quantize", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("gmm_prepare_quantized_host", ctypes.c_int,
     [ctypes.POINTER(MixtureSetDesc), ctypes.c_int, _f32p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
      ctypes.c_void_p]),
    ("gmm_scorer_launch_info", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint32, _u32p, ctypes.POINTER(ctypes.c_char_p)]),
    ("gmm_scorer_set_timing", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("gmm_scorer_kernel_time", ctypes.c_int,
     [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), _u32p, ctypes.c_int]),
    ("gmm_scorer_density_clustering", ctypes.c_int,
     [ctypes.c_void_p, _u32p, _u32p, ctypes.c_void_p, ctypes.c_void_p]),
    ("gmm_scorer_cluster_selection", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]),
    ("gmm_scorer_clustering_source", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
    ("gmm_cache_archive_read_item", ctypes.c_int,
     [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
    ("gmm_cache_archive_write_item", ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_uint64]),
    ("gmm_density_clustering_seeds", ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, _u32p]),
    ("gmm_shard_pack_keys", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
      ctypes.c_void_p, ctypes.c_void_p]),
    ("gmm_shard_unpack_keys", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
      ctypes.c_void_p]),
    ("gmm_density_shard_plan", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, _u32p]),
    ("gmm_scorer_create_sharded", ctypes.c_int,
     [ctypes.POINTER(MixtureSetDesc), ctypes.c_int, ctypes.POINTER(ScorerConfig), ctypes.c_void_p, ctypes.c_uint32,
      ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    ("gmm_scorer_shard_info", ctypes.c_int, [ctypes.c_void_p, _u32p, ctypes.POINTER(ctypes.c_int)]),
    ("gmm_last_error", ctypes.c_char_p, []),
    # include/rasr_gmm_io.h
    ("gmm_mixture_set_read", ctypes.c_int,
     [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(MixtureSetDesc)]),
    ("gmm_mixture_set_parse", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(MixtureSetDesc)]),
    ("gmm_mixture_set_free", ctypes.c_int, [ctypes.POINTER(MixtureSetDesc)]),
    ("gmm_default_estimator_config", None, [ctypes.POINTER(EstimatorConfig)]),
    ("gmm_mixture_set_estimate", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(EstimatorConfig), ctypes.POINTER(MixtureSetDesc)]),
    ("gmm_mixture_set_read_config", ctypes.c_int,
     [ctypes.c_char_p, ctypes.POINTER(EstimatorConfig), ctypes.c_uint32, ctypes.c_uint32,
      ctypes.POINTER(MixtureSetDesc)]),
    ("gmm_mixture_set_write", ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(MixtureSetDesc), ctypes.c_uint32]),
    ("gmm_version", ctypes.c_char_p, []),
    ("gmm_kernel_id", ctypes.c_char_p, []),
]

_lib = None


def load_library(path: str | None = None) -> ctypes.CDLL:
    """Load librasr_gmm.so (raises if it has not been built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(
            f"rasr_amd native library not found at {p}: the MI355X scorer has no fallback; "
            "build it with `make` (or __graft_entry__.build())")
    # Two HIP runtimes end up in a Python process: the image's ROCm (librasr_gmm.so's libamdhip64.so.7)
    # and the one bundled with torch.  When librasr_gmm.so is loaded before torch, torch's HIP calls partly
    # bind to the ROCm copy and, once torch has initialised the device, hipGetDeviceCount in the ROCm copy
    # fails ("no HIP device available"; scripts/debug/probe_order.py).  Loading torch first keeps each
    # library on its own runtime.  (C++ callers such as RASR have one runtime and are unaffected.)
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(p)
    for name, res, args in PROTOTYPES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


class GmmError(RuntimeError):
    pass


def check(rc: int, what: str = "") -> None:
    if rc != GMM_OK:
        msg = load_library().gmm_last_error()
        raise GmmError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
