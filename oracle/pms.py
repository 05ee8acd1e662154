"""TEST INFRASTRUCTURE ONLY -- ctypes binding of oracle/_build/libpms_oracle.so, the
std::istream restatement of RASR's mixture-set text reader (oracle/pms_istream.cc).

It uses the same libstdc++ extraction operators as the reference's MixtureSet::read
(src/Mm/MixtureSet.cc:170-214), so it pins the product's own tokenizer.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .oracle import OrcMixtureSet, build

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "_build", "libpms_oracle.so")
_lib = None

# return codes of orc_pms_read
OK, STREAM_FAIL, VERSION, COVARIANCE_TYPE, SHORT_HEADER = 0, 1, 2, 3, 4


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        _lib.orc_pms_read.restype = ctypes.c_int
        _lib.orc_pms_read.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.POINTER(OrcMixtureSet)]
        _lib.orc_pms_free.restype = None
        _lib.orc_pms_free.argtypes = [ctypes.POINTER(OrcMixtureSet)]
    return _lib


def pms_read(path: str, dimension_offset: int = 0, reduced_dimension: int = 0):
    """(status, tables) -- tables is a dict of numpy arrays (None unless status == OK)."""
    lib = _load()
    d = OrcMixtureSet()
    rc = lib.orc_pms_read(os.fsencode(path), dimension_offset, reduced_dimension, ctypes.byref(d))
    if rc != OK:
        return rc, None
    try:
        def arr(ptr, n, dt):
            return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dt, copy=True) if n else np.zeros(0, dt)
        D = d.dimension
        n_entries = d.mixture_offsets[d.n_mixtures]
        return rc, {
            "means": arr(d.means, d.n_means * D, np.float32).reshape(d.n_means, D),
            "variances": arr(d.variances, d.n_covariances * D, np.float32).reshape(d.n_covariances, D),
            "density_mean": arr(d.density_mean, d.n_densities, np.uint32),
            "density_covariance": arr(d.density_covariance, d.n_densities, np.uint32),
            "mixture_offsets": arr(d.mixture_offsets, d.n_mixtures + 1, np.uint32),
            "mixture_densities": arr(d.mixture_densities, n_entries, np.uint32),
            "mixture_log_weights": arr(d.mixture_log_weights, n_entries, np.float64),
        }
    finally:
        lib.orc_pms_free(ctypes.byref(d))
