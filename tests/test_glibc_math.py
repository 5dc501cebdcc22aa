"""glibc_math.h's restatements of glibc 2.35 (cbrt, hypot, clog's real part) against the host's glibc,
bit for bit. The reference's AP3P quartic (ap3p.cpp:10-59) calls these through libstdc++; the GPU kernel
runs the restatements, so these tests pin the device's cbrt / hypot bits to glibc's. CPU only."""
import numpy as np
import pytest

from minicv_amd import native as N


def _ours(fn, a, b=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(a if b is None else b, dtype=np.float64)
    out = np.zeros_like(a)
    assert N.lib().mcvHostGlibcMath(fn, a.ctypes.data, b.ctypes.data, a.shape[0], out.ctypes.data) == a.shape[0]
    return out


def _bits_equal(x, y):
    return np.array_equal(x.view(np.uint64), y.view(np.uint64))


def _random_doubles(rng, n):
    """Random bit patterns (every exponent, subnormals, signs) minus non-finite ones, plus the ranges the
    AP3P quartic meets (magnitudes 1e-12 .. 1e12) and exact cubes / powers of two."""
    raw = rng.integers(0, 2**64, size=n, dtype=np.uint64).view(np.float64)
    raw = raw[np.isfinite(raw)]
    mid = rng.uniform(-1, 1, n) * 10.0 ** rng.uniform(-12, 12, n)
    cubes = rng.integers(-10**5, 10**5, n // 10).astype(np.float64) ** 3
    pows = 2.0 ** rng.integers(-1074, 1023, n // 10).astype(np.float64)
    special = np.array([0.0, -0.0, 1.0, -1.0, 8.0, -27.0, 5e-324, -5e-324, 1.7976931348623157e308, 2.2250738585072014e-308])
    return np.concatenate([raw, mid, cubes, pows, special])


def test_cbrt_equals_glibc(native, oracle):
    rng = np.random.default_rng(1)
    for _ in range(4):
        x = _random_doubles(rng, 500_000)
        ref = oracle.libm(0, x)
        got = _ours(0, x)
        bad = np.nonzero(got.view(np.uint64) != ref.view(np.uint64))[0]
        assert len(bad) == 0, f"{len(bad)} mismatches, e.g. cbrt({x[bad[0]]!r}) = {got[bad[0]]!r} vs {ref[bad[0]]!r}"
    assert _bits_equal(_ours(0, np.array([np.inf, -np.inf])), oracle.libm(0, np.array([np.inf, -np.inf])))
    assert np.isnan(_ours(0, np.array([np.nan]))).all()


def test_hypot_equals_glibc(native, oracle):
    rng = np.random.default_rng(2)
    for _ in range(4):
        a = _random_doubles(rng, 300_000)
        b = rng.permutation(_random_doubles(rng, 300_000))[:a.shape[0]]
        a = a[:b.shape[0]]
        # near-equal magnitudes and the scaling thresholds (2^511, 2^-511, ratio 2^54)
        c = rng.uniform(0.5, 2, 50_000) * 2.0 ** rng.integers(-600, 600, 50_000)
        d = c * rng.uniform(0.999, 1.001, 50_000) * rng.choice([1.0, 2.0 ** -54, 2.0 ** -53, 2.0 ** 27], 50_000)
        a, b = np.concatenate([a, c]), np.concatenate([b, d])
        ref = oracle.libm(1, a, b)
        got = _ours(1, a, b)
        bad = np.nonzero(got.view(np.uint64) != ref.view(np.uint64))[0]
        assert len(bad) == 0, f"{len(bad)} mismatches, e.g. hypot({a[bad[0]]!r}, {b[bad[0]]!r})"


def test_clog_real_part_equals_glibc(native, oracle):
    """The host twin of glibc_clog_re (host libm's log / log1p) equals glibc's clog real part: the branch
    structure and __x2y2m1 are glibc's. Arguments cluster where the branches differ (|z| in [0.5, 2),
    near 1, |y| around DBL_EPSILON, huge and tiny)."""
    rng = np.random.default_rng(3)
    n = 400_000
    r = 1.0 + rng.normal(size=n) * 10.0 ** rng.uniform(-17, 0, n)
    th = rng.uniform(-np.pi, np.pi, n)
    a, b = r * np.cos(th), r * np.sin(th)
    a2 = rng.uniform(0.5, 2, n) * rng.choice([1, -1], n)
    b2 = rng.uniform(0, 1, n) * 10.0 ** rng.uniform(-18, 0, n) * rng.choice([1, -1], n)
    a3 = _random_doubles(rng, n)[:n]
    b3 = _random_doubles(rng, n)[:n]
    ones = np.ones(1000) * rng.choice([1, -1], 1000)
    b4 = rng.normal(size=1000) * 10.0 ** rng.uniform(-10, 0, 1000)
    A = np.concatenate([a, a2, b2, a3, ones])
    B = np.concatenate([b, b2, a2, b3, b4])
    keep = ~((A == 0) & (B == 0))
    A, B = A[keep], B[keep]
    ref = oracle.libm(2, A, B)
    got = _ours(2, A, B)
    bad = np.nonzero(got.view(np.uint64) != ref.view(np.uint64))[0]
    assert len(bad) == 0, f"{len(bad)} mismatches, e.g. clog({A[bad[0]]!r} + i {B[bad[0]]!r}).real"
