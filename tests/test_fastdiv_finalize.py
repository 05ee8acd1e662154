"""The SIMD-diagonal-maximum finalize (SimdFeatureScorer.cc:142: (f32)(0.5 * q / (f64) scalingSquared_)) as
the quantized kernel computes it (gmm_kernels_i8.hip, emitMixtureI8, GMM_I8_FASTDIV): y = q * 0.5 RN64(1/s2)
in double, (f32) y unless the 29 bits below f32 precision lie within 4 of the rounding midpoint 2^28, else
the division.  Restated in numpy (IEEE double multiply and round-to-nearest conversions, as the GPU's
v_mul_f64 / v_cvt_f32_f64) and checked bit for bit against the division on random and adversarial inputs."""
import numpy as np


def _exact(q, s2):
    return (0.5 * q.astype(np.float64) / s2.astype(np.float64)).astype(np.float32)


def _fast(q, s2):
    hr = 0.5 * (1.0 / s2.astype(np.float64))
    y = q.astype(np.float64) * hr
    lo = (y.view(np.uint64) & np.uint64(0x1FFFFFFF)).astype(np.int64)
    near = np.abs(lo - (1 << 28)) <= 4
    return np.where(near, _exact(q, s2), y.astype(np.float32)), near


def test_random_scores_bit_exact():
    rng = np.random.default_rng(7)
    n = 4_000_000
    q = rng.integers(-(2**31), 2**31 - 1, n, dtype=np.int64)
    q[::2] = rng.integers(-20000, 3_000_000, len(q[::2]))  # the range real minima take
    s2 = rng.uniform(1.0, 4000.0, n).astype(np.float32)
    s2[::7] = (1.0 / rng.uniform(1e-3, 10.0, len(s2[::7]))).astype(np.float32)
    f, _ = _fast(q, s2)
    assert np.array_equal(f.view(np.uint32), _exact(q, s2).view(np.uint32))


def test_midpoint_neighbourhood_takes_the_division():
    """Quotients placed on and around f32 rounding midpoints: the guard must catch every one that the
    multiplication would round differently, and the result must equal the division everywhere."""
    rng = np.random.default_rng(8)
    s2 = rng.uniform(1.0, 4000.0, 200_000).astype(np.float32)
    # q such that 0.5 q / s2 is close to a midpoint m = (f + ulp/2): q = round(2 m s2)
    f = rng.uniform(1.0, 1e5, len(s2)).astype(np.float32)
    ulp = np.spacing(f).astype(np.float64)
    m = f.astype(np.float64) + ulp / 2
    q = np.rint(2.0 * m * s2.astype(np.float64)).astype(np.int64)
    q = np.clip(q, -(2**31), 2**31 - 1)
    out, near = _fast(q, s2)
    assert np.array_equal(out.view(np.uint32), _exact(q, s2).view(np.uint32))
    y = q.astype(np.float64) * (0.5 * (1.0 / s2.astype(np.float64)))
    wrong = y.astype(np.float32).view(np.uint32) != _exact(q, s2).view(np.uint32)
    assert not (wrong & ~near).any()  # every case the multiplication alone gets wrong is guarded
