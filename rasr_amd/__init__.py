"""rasr_amd -- MI355X-native diagonal-GMM acoustic scorer behind RASR's
Mm::FeatureScorer plugin surface.

The product is the C-ABI library rasr_amd/lib/librasr_gmm.so (HIP kernels for
gfx950 + host-side model preparation); this package only binds it.
"""
from ._capi import (BATCH_DIAGONAL_MAXIMUM_FAST, BATCH_DIAGONAL_MAXIMUM_FLOAT, BATCH_DIAGONAL_MAXIMUM_INT,
                    DIAGONAL_MAXIMUM, LIB_PATH, SCORER_TYPES, SIMD_DIAGONAL_MAXIMUM, GmmError, load_library)
from .mixture_set import (MixtureSet, estimate_mixture_set, estimator_config, parse_mixture_set, ragged_counts,
                          read_mixture_set, synthetic_frames,
                          synthetic_mixture_set, write_mixture_set)
from .scorer import Scorer, default_config, pinned_empty, prepare_quantized_host

__all__ = [
    "BATCH_DIAGONAL_MAXIMUM_FAST", "BATCH_DIAGONAL_MAXIMUM_FLOAT", "BATCH_DIAGONAL_MAXIMUM_INT", "DIAGONAL_MAXIMUM",
    "SIMD_DIAGONAL_MAXIMUM", "SCORER_TYPES", "LIB_PATH", "GmmError", "load_library", "MixtureSet", "ragged_counts",
    "synthetic_frames", "synthetic_mixture_set", "Scorer", "default_config", "pinned_empty", "prepare_quantized_host",
    "read_mixture_set", "parse_mixture_set", "write_mixture_set", "estimate_mixture_set", "estimator_config",
]
