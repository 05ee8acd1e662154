"""The C-ABI library loads, exports every function include/*.h declares, and reports
errors as status codes (no compute call needs a GPU here)."""
import ctypes
import glob
import os
import re

import pytest

import rasr_amd as ra
from rasr_amd import _capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    names = []
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\*?\s+\**\s*((?:gmm|nn)_[a-z0-9_]+)\s*\(",
                             src, re.M):
            names.append(m.group(1))
    return sorted(set(names))


def test_header_declares_api():
    names = _declared_functions()
    assert "gmm_scorer_create" in names and "gmm_score_device" in names and len(names) >= 15
    assert "nn_scorer_create" in names and "nn_score_device" in names  # include/rasr_nn.h


def test_library_exports_every_declared_symbol(built):
    from rasr_amd import nn
    lib = ctypes.CDLL(_capi.LIB_PATH)
    missing = [n for n in _declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    bound = {p[0] for p in _capi.PROTOTYPES} | {p[0] for p in nn._PROTOTYPES}
    assert set(_declared_functions()) <= bound, set(_declared_functions()) - bound


def test_nn_errors_without_device(built):
    from rasr_amd import nn
    lib = nn._lib()
    h = ctypes.c_void_p()
    assert lib.nn_scorer_create(None, 4, 0, ctypes.byref(h)) == -1
    assert lib.nn_score_device(None, None, 1, 8, None, 1, None) == -1
    assert lib.nn_scorer_destroy(None) == 0


def test_library_is_native_gfx950(built):
    # the shared object carries a gfx950 code object (no CPU fallback inside)
    data = open(_capi.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    assert b"scoreI8" in data and b"scoreF32" in data


def test_default_config_and_version(built):
    cfg = ra.default_config()
    assert cfg.mixture_weight_scale == 1.0 and cfg.gaussian_scale == 1.0 and cfg.score_scale == 1.0
    assert cfg.max_frames == 4  # "buffer-size" default (BatchFeatureScorer.cc:28-29)
    assert b"gfx950" in ra.load_library().gmm_version()


def test_error_codes_without_device(built):
    lib = ra.load_library()
    h = ctypes.c_void_p()
    assert lib.gmm_scorer_create(None, 9, None, 0, ctypes.byref(h)) == -1
    assert b"null" in lib.gmm_last_error()
    ms = ra.synthetic_mixture_set(3, 2, 8, seed=1)
    d = ms.desc()
    assert lib.gmm_scorer_create(ctypes.byref(d), 77, None, 0, ctypes.byref(h)) == -2  # unknown type
    assert lib.gmm_score_device(None, None, 1, 8, None, None, 1, None) == -1
    assert lib.gmm_scorer_destroy(None) == 0


def test_fast_type_dimension_limit(built):
    # batch-diagonal-maximum-fast supports padded dimension <= 48 (BatchFeatureScorer.cc:552-556)
    lib = ra.load_library()
    ms = ra.synthetic_mixture_set(3, 2, 50, seed=1)
    d = ms.desc()
    h = ctypes.c_void_p()
    assert lib.gmm_scorer_create(ctypes.byref(d), 4, None, 0, ctypes.byref(h)) == -2
    assert b"48" in lib.gmm_last_error()


def test_product_path_has_no_oracle_dependency():
    # the product package must not import or link the test oracle
    for f in glob.glob(os.path.join(ROOT, "rasr_amd", "**", "*.*"), recursive=True):
        if f.endswith((".py", ".cc", ".hh", ".hip", ".h")):
            src = open(f).read()
            assert "import oracle" not in src and "gmm_oracle" not in src and "libgmm_oracle" not in src, f
