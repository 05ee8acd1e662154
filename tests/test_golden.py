"""Frozen vectors (tests/golden, made by scripts/make_golden.py from the oracle).

They guard the oracle and the product's host preparation against regressions
(CPU) and are a second, data-only parity target for the GPU path.  Tables that
depend on the host CPU's rsqrtss (the reference's -ffast-math 1/sqrt) are
checked first; on a CPU whose rsqrtss differs the fixture is skipped."""
import glob
import os

import numpy as np
import pytest

import oracle
import rasr_amd as ra

# tests/golden/*.npz: made in the build container; tests/golden/cpu_*/*.npz: the same cases made by the
# oracle on another host CPU (its rsqrtss), e.g. the GPU box's (scripts/make_golden.py --out)
GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz")) +
                glob.glob(os.path.join(os.path.dirname(__file__), "golden", "cpu_*", "*.npz")))


def _load(path):
    z = np.load(path, allow_pickle=False)
    ms = ra.MixtureSet(z["means"], z["variances"], z["density_mean"], z["density_covariance"], z["mixture_offsets"],
                       z["mixture_densities"], z["mixture_log_weights"])
    return ms, z


def _same_rsqrt(ms, z):
    o = oracle.OracleSimd(ms)
    if not np.array_equal(o.isv, z["simd_isv"]):
        pytest.skip(f"host rsqrtss differs from the fixture's ({z['cpu_vendor']})")
    return o


def test_golden_present():
    assert len(GOLDEN) >= 4


@pytest.mark.parametrize("path", GOLDEN, ids=os.path.basename)
def test_oracle_reproduces_golden(path):
    ms, z = _load(path)
    o = _same_rsqrt(ms, z)
    s, b, raw = o.score(z["frames"])
    assert np.array_equal(s.view(np.uint32), z["simd_scores"].view(np.uint32))
    assert np.array_equal(b, z["simd_best"]) and np.array_equal(raw, z["simd_raw"])
    fs, fb = oracle.OracleFloat(ms).score(z["frames"])
    assert np.array_equal(fs.view(np.uint32), z["float_scores"].view(np.uint32))
    assert np.array_equal(fb, z["float_best"])
    if "batch_int_scores" in z:
        assert np.array_equal(oracle.batch_int_score(ms, z["frames"]), z["batch_int_scores"])
        assert np.array_equal(oracle.batch_float_score(ms, z["frames"]), z["batch_float_scores"])


@pytest.mark.parametrize("path", GOLDEN, ids=os.path.basename)
def test_host_prep_matches_golden(built, path):
    ms, z = _load(path)
    _same_rsqrt(ms, z)
    p = ra.prepare_quantized_host(ms)
    assert p["scaling"] == float(z["simd_scaling"])
    assert np.array_equal(p["prepared_mean"], z["simd_prepared_mean"])
    assert np.array_equal(p["constant_weight"], z["simd_constant_weight"])


@pytest.mark.gpu
@pytest.mark.parametrize("path", GOLDEN, ids=os.path.basename)
def test_gpu_matches_golden(gpu, path):
    ms, z = _load(path)
    _same_rsqrt(ms, z)
    frames = z["frames"]
    s, b = ra.Scorer(ms, "SIMD-diagonal-maximum", max_frames=len(frames)).score_host(frames)
    assert np.array_equal(s.view(np.uint32), z["simd_scores"].view(np.uint32))
    assert np.array_equal(b, z["simd_best"])
    fs, fb = ra.Scorer(ms, "diagonal-maximum", max_frames=len(frames)).score_host(frames)
    ref = z["float_scores"].astype(np.float64)
    assert (np.abs(fs - ref) / np.maximum(1, np.abs(ref))).max() <= 1e-4
    if "batch_int_scores" in z:
        bs, _ = ra.Scorer(ms, "batch-diagonal-maximum-int", max_frames=len(frames)).score_host(frames)
        assert np.array_equal(bs.view(np.uint32), z["batch_int_scores"].view(np.uint32))
