"""The quantized scorers' finalize as the kernels compute it (gmm_kernels_i8.hip finalizeStoreI8): both reference
finalizes divide by b = 2 s^2 -- SIMD-diagonal-maximum (f32)(0.5 * q / (f64) scalingSquared_) (SimdFeatureScorer.cc:142)
and batch-diagonal-maximum-int (f32)best / scale_ (BatchFeatureScorer.cc:468, scale_ = 2 s^2) -- and the kernel forms
y = RN(x / b) from x (rh + rl) -- 1/b as two floats, a faithful quotient -- and one Markstein correction, the SIMD
scorer for |q| < 2^24 only (larger |q| divide in double).  Restated with every f32 operation rounded once from its exact value (fractions) and checked bit for bit
against the references' own arithmetic (numpy IEEE division) on random and adversarial inputs."""
import numpy as np
from fractions import Fraction


def _rn32(v: Fraction) -> np.float32:
    """v rounded to the nearest f32, ties to even (no overflow / subnormals in this range)."""
    c = np.float32(float(v))
    best = None
    for cand in (np.nextafter(c, np.float32(-np.inf)), c, np.nextafter(c, np.float32(np.inf))):
        d = abs(Fraction(float(cand)) - v)
        if best is None or d < best[0] or (d == best[0] and int(cand.view(np.uint32)) % 2 == 0):
            best = (d, cand)
    return best[1]


def _markstein(q: int, b: np.float32) -> np.float32:
    """The kernel's sequence: rh = RN(1/b) (IEEE f32 division), rl = RN(1/b - rh) (host, in double),
    y = fma(x, rh, RN(x rl)), then y + fma(-b, y, x) rh in one more fma."""
    x = np.float32(q)
    rh = np.float32(1.0) / b
    rl = np.float32(1.0 / float(b) - float(rh))
    fx, fb, fr = Fraction(float(x)), Fraction(float(b)), Fraction(float(rh))
    y = _rn32(fx * fr + Fraction(float(_rn32(fx * Fraction(float(rl))))))
    e = _rn32(fx - fb * Fraction(float(y)))
    return _rn32(Fraction(float(e)) * fr + Fraction(float(y)))


def _simd_reference(q: int, s2: np.float32) -> np.float32:
    return np.float32(0.5 * float(q) / float(s2))  # SimdFeatureScorer.cc:142, double then f32


def test_simd_finalize_random():
    rng = np.random.default_rng(7)
    s2 = rng.uniform(1.0, 4000.0, 20000).astype(np.float32)
    s2[::7] = (1.0 / rng.uniform(1e-3, 10.0, len(s2[::7]))).astype(np.float32)
    q = rng.integers(-(2**24) + 1, 2**24, len(s2))
    q[::2] = rng.integers(-20000, 3_000_000, len(q[::2]))  # the range real minima take
    for qi, si in zip(q.tolist(), s2):
        b = np.float32(2.0) * si  # exact
        assert _markstein(qi, b).view(np.uint32) == _simd_reference(qi, si).view(np.uint32), (qi, float(si))


def test_simd_finalize_midpoints():
    """Quotients on and next to f32 rounding midpoints, where a double rounding or a plain product could differ."""
    rng = np.random.default_rng(8)
    hits = 0
    for _ in range(8000):
        s2 = np.float32(rng.uniform(1.0, 4000.0))
        f = np.float32(rng.uniform(1.0, 1e5))
        m = Fraction(float(f)) + Fraction(float(np.spacing(f))) / 2
        q = int(round(m * 2 * Fraction(float(s2))))
        if abs(q) >= 2**24:
            continue
        b = np.float32(2.0) * s2
        want = _simd_reference(q, s2)
        assert _markstein(q, b).view(np.uint32) == want.view(np.uint32), (q, float(s2))
        hits += int((np.float32(q) * (np.float32(1.0) / b)).view(np.uint32) != want.view(np.uint32))
    assert hits > 0  # hard cases: the plain product misses some of them


# ---------------------------------------------------------------------------------------------------------------
# batch-diagonal-maximum-int / -fast finalize (BatchFeatureScorer.cc:468: (f32)best / scale_) as the kernels compute
# it (gmm_kernels_i8.hip finalizeStoreI8): x = (f32) q, rh = RN(1 / b), rl = RN(1 / b - rh) from the host,
# y = fma(x, rh, RN(x rl)), then y = fma(fma(-b, y, x), rh, y).  Restated with every f32 operation rounded once from its exact value (fractions),
# checked against the correctly rounded quotient RN(x / b) -- random integers over the whole int32 range and the
# real minima's range, and quotients placed on and next to f32 rounding midpoints.
# ---------------------------------------------------------------------------------------------------------------
def _batch_cases(n, seed):
    rng = np.random.default_rng(seed)
    b = (2.0 * rng.uniform(1.0, 4000.0, n) ** 1).astype(np.float32)  # scale_ = 2 s^2
    q = rng.integers(-(2**31), 2**31 - 1, n, dtype=np.int64)
    q[::2] = rng.integers(-20000, 3_000_000, len(q[::2]))
    return q, b


def test_batch_finalize_markstein_random():
    q, b = _batch_cases(20000, 11)
    for qi, bi in zip(q.tolist(), b):
        want = np.float32(qi) / bi  # numpy f32 division: correctly rounded
        got = _markstein(qi, bi)
        assert got.view(np.uint32) == want.view(np.uint32), (qi, float(bi))


def test_batch_finalize_markstein_midpoints():
    """x / b within a few units of 2^-40 relative of an f32 midpoint: where a plain x * RN(1/b) goes wrong."""
    rng = np.random.default_rng(12)
    hits = 0
    for _ in range(6000):
        b = np.float32(2.0 * rng.uniform(1.0, 4000.0))
        f = np.float32(rng.uniform(1.0, 2e6))
        m = Fraction(float(f)) + Fraction(float(np.spacing(f))) / 2  # midpoint above f
        q = int(round(m * Fraction(float(b))))
        if abs(q) >= 2**24:  # (f32) q must be q itself for the quotient to sit at the midpoint
            continue
        x = np.float32(q)
        want = x / b
        assert _markstein(q, b).view(np.uint32) == want.view(np.uint32), (q, float(b))
        hits += int((x * (np.float32(1.0) / b)).view(np.uint32) != want.view(np.uint32))
    assert hits > 0  # the cases are hard: the plain product misses some of them
