"""Known-answer tests for the oracle's scalar arithmetic, derived by hand from the
reference source (the reference has no tests or fixtures for src/Mm).

Each expectation cites the reference expression and the effect of its build flags
(-O2 -ffast-math -msse3, config/cc-gcc.make, config/proc-x86_64.make)."""
import math

import numpy as np
import pytest

import oracle


def f32(x):
    return float(np.float32(x))


def test_quantize_round_half_away_and_clip():
    # quantize<f32,u8> (Utilities.hh:186-190): clip((int)round(x) + 128, 0, 255)
    xs = [0.0, 0.5, -0.5, 1.5, 2.5, -2.5, 0.49999997, -0.49999997, 126.5, 127.49998, 127.5, -127.5,
          -128.4, -128.5, 1000.0, -1000.0]
    want = [128, 129, 127, 130, 131, 125, 128, 128, 255, 255, 255, 0, 0, 0, 255, 0]
    assert list(oracle.quantize_array(xs)) == want


def test_quantize_x86_conversion_quirks():
    # (int)round(x) is cvttss2si: out-of-range and NaN give 0x80000000; +128 then clips to 0.
    # 2147483520 (largest float below 2^31) + 128 wraps to INT_MIN in the 32-bit add, then clips to 0.
    got = oracle.quantize_array([3e9, -3e9, float("nan"), float("inf"), 2147483520.0, 2.1e9])
    assert list(got) == [0, 0, 0, 0, 0, 255]


def test_quantize_matches_round_half_away_dense():
    # GCC's fast-math round expansion (add nextbelow(0.5) with sign, truncate) equals
    # round-half-away-from-zero on every float of the quantizer's working range.
    rng = np.random.default_rng(0)
    x = np.concatenate([
        rng.uniform(-200, 200, 2_000_000).astype(np.float32),
        (np.arange(-400, 401) / 2).astype(np.float32),                       # exact halves
        np.nextafter((np.arange(-400, 401) / 2).astype(np.float32), np.float32(np.inf)),
        np.nextafter((np.arange(-400, 401) / 2).astype(np.float32), np.float32(-np.inf)),
    ])
    xd = x.astype(np.float64)
    r = np.where(xd >= 0, np.floor(xd + 0.5), -np.floor(-xd + 0.5))
    want = np.clip(r + 128, 0, 255).astype(np.uint8)
    assert np.array_equal(oracle.quantize_array(x), want)


@pytest.mark.parametrize("v", [0.5, 1.0, 2.0, 4.0, 0.7321, 1.9, 3.14159, 123.456])
def test_inverse_sqrt_newton_raphson(v):
    # inverseSquareRoot<f32> under -ffast-math: rsqrtss + one Newton step -> ~1e-7 relative, not exact
    got = oracle.inverse_sqrt(v)
    assert abs(got - 1 / math.sqrt(v)) <= 2e-7 * (1 / math.sqrt(v))


def test_gauss_log_norm_sequential_double():
    # gaussLogNormFactor (Utilities.hh:55-76): D*log(2 pi) + sum log|v|, double, in order
    v = np.array([0.5, 1.25, 3.0, 0.75, 2.2], dtype=np.float32)
    acc = 0.0
    for x in v:
        acc += math.log(abs(float(x)))
    want = len(v) * math.log(2 * math.pi) + acc
    assert oracle.gauss_log_norm(v) == want


def test_quantization_scaling_factor_single_precision():
    # quantizationScalingFactor (SimdFeatureScorer.cc:128-133) folds to 102.0f / max|.| in f32
    for lo, hi in [(-3.0, 2.5), (-1.7, 4.2), (-0.3, 0.2), (-5.123, -0.5)]:
        m = np.float32(max(abs(lo), abs(hi)))
        assert oracle.quantization_scaling_factor(lo, hi) == f32(np.float32(102.0) / m)


def test_constant_weight_rounding_chain():
    # SimdFeatureScorer.cc:96 + IntelOptimization.cc:47:
    #   (s32)((f32)((f64)(s2 * -2.0f) * logw) + logNorm_f32), truncation toward zero
    for s2, lw, ln in [(400.0, math.log(1 / 160), 17000.5), (123.25, -7.3, -250.75), (1.0, -0.1, 0.3),
                       (55.5, math.log(0.3), -12.9)]:
        w = np.float32(float(np.float32(s2) * np.float32(-2.0)) * lw)
        total = np.float32(w + np.float32(ln))
        assert oracle.constant_weight(s2, lw, ln) == int(math.trunc(float(total)))


def test_simd_final_score_double_path():
    # SimdFeatureScorer.cc:142: (f32)(0.5 * q / (double)s2)
    for q, s2 in [(12345, 400.0), (-17, 3.5), (2147483647, 421.87), (0, 1.0)]:
        assert oracle.simd_final_score(q, s2) == f32(0.5 * q / float(np.float32(s2)))


def test_float_distance_sse3_order():
    # GaussDiagonalMaximumFeatureScorer::distance, SSE3 path: 4-lane partial sums, hadd, scalar tail
    rng = np.random.default_rng(3)
    for d in (39, 45, 4, 5, 7):
        f = rng.standard_normal(d).astype(np.float32)
        m = rng.standard_normal(d).astype(np.float32)
        s = (1 + rng.random(d)).astype(np.float32)
        df = ((m - f) * s).astype(np.float32)
        sq = (df * df).astype(np.float32)
        eff = d & ~3
        lanes = np.zeros(4, np.float32)
        for i in range(0, eff, 4):
            lanes = (lanes + sq[i:i + 4]).astype(np.float32)
        r = np.float32(np.float32(0) + np.float32(np.float32(lanes[0] + lanes[1]) + np.float32(lanes[2] + lanes[3])))
        for i in range(eff, d):
            r = np.float32(r + sq[i])
        assert oracle.float_distance(f, m, s) == float(r)
