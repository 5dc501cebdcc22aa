"""glibc_math.h's restatements of glibc 2.35 (cbrt, hypot, clog's real part, exp, log, log1p, cos,
atan2) against the host's glibc, bit for bit. The reference's AP3P quartic (ap3p.cpp:10-59) calls these
through libstdc++ (std::cbrt, the complex sqrt and pow); the GPU kernel runs the restatements, so these
tests pin the device's bits to glibc's. CPU only."""
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


def _check(oracle, fn, a, b=None, name=""):
    ref = oracle.libm(fn, a, a if b is None else b)
    got = _ours(fn, a, b)
    bad = np.nonzero(got.view(np.uint64) != ref.view(np.uint64))[0]
    assert len(bad) == 0, (f"{len(bad)} mismatches of {len(a)}, e.g. {name}({a[bad[0]]!r}"
                           + ("" if b is None else f", {b[bad[0]]!r}") + f") = {got[bad[0]]!r} vs {ref[bad[0]]!r}")


def test_exp_equals_glibc(native, oracle):
    """exp over |x| < 512 (glibc_exp's domain; AP3P feeds it log|w| / 3): uniform, small |x| near the
    2^-54 cut, multiples of ln2 / 128 (the table's nodes) and their neighbours."""
    rng = np.random.default_rng(4)
    n = 400_000
    x = np.concatenate([
        rng.uniform(-511, 511, n),
        rng.uniform(-1, 1, n) * 10.0 ** rng.uniform(-20, 0, n),
        (rng.integers(-20000, 20000, n) * (np.log(2) / 128)) * (1 + rng.choice([-1, 0, 1], n) * 2.0 ** -52),
        np.array([0.0, -0.0, 2.0 ** -54, -2.0 ** -54, 2.0 ** -55, 1.0, -1.0, 511.0, -511.0]),
    ])
    _check(oracle, 4, x, name="exp")


def test_log_equals_glibc(native, oracle):
    """log over positive normal and subnormal x outside glibc's close-to-1 band [1 - 2^-4, 1 + 0x1.09p-4)
    (the band clog never sends to log)."""
    rng = np.random.default_rng(5)
    n = 400_000
    x = np.concatenate([
        10.0 ** rng.uniform(-307, 308, n),
        np.abs(_random_doubles(rng, n)),
        rng.uniform(0.5, 2.0, n),
        2.0 ** rng.integers(-1074, 1024, n // 10).astype(np.float64),
        np.array([np.inf]),
    ])
    lo, hi = 1 - 2.0 ** -4, 1 + float.fromhex("0x1.09p-4")
    x = x[(x > 0) & ~((x >= lo) & (x < hi))]
    _check(oracle, 5, x, name="log")


def test_log1p_equals_glibc(native, oracle):
    """log1p over x > -1: every magnitude, the branch cuts of s_log1p.c (|x| < 2^-29, 2^-54, the
    sqrt(2) / 2 - 1 and sqrt(2) - 1 boundaries, 2^53) and clog's x^2 + y^2 - 1 range [-0.5, 3)."""
    rng = np.random.default_rng(6)
    n = 400_000
    x = np.concatenate([
        _random_doubles(rng, n),
        rng.uniform(-0.5, 3.0, n),
        rng.uniform(-1, 1, n) * 10.0 ** rng.uniform(-20, 0, n),
        np.array([-0.2928932188134524, -0.29289321881345254, 0.41421356237309503, 0.41421356237309515,
                  2.0 ** -29, 2.0 ** -54, 2.0 ** 53, -0.9999999999999999]),
    ])
    cuts = np.array([-0.2928932188134524, 0.41421356237309503, 2.0 ** -29, 2.0 ** -54, 2.0 ** 53])
    x = np.concatenate([x, (cuts[:, None] * (1 + np.arange(-64, 65) * 2.0 ** -52)).ravel()])
    x = x[x > -1]
    _check(oracle, 6, x, name="log1p")


def test_cos_equals_glibc(native, oracle):
    """cos over |x| <= pi / 2 - 0.126 (glibc_cos's domain; AP3P feeds it arg(w) / 3, |.| <= pi / 3):
    uniform, the 0.855469 switch to sin(pi / 2 - |x|), tiny |x| and the table nodes i / 128."""
    rng = np.random.default_rng(7)
    n = 400_000
    x = np.concatenate([
        rng.uniform(-1.4447, 1.4447, n),
        rng.uniform(-1, 1, n) * 10.0 ** rng.uniform(-12, 0, n),
        0.855469 * (1 + rng.integers(-1000, 1000, n // 10) * 2.0 ** -52),
        rng.integers(-184, 185, n // 10) / 128.0 * (1 + rng.choice([-1, 0, 1], n // 10) * 2.0 ** -52),
        np.array([0.0, -0.0, np.pi / 3, -np.pi / 3, 2.0 ** -27, 2.0 ** -28]),
    ])
    _check(oracle, 7, x, name="cos")


def test_atan2_equals_glibc(native, oracle):
    """atan2 over every quadrant with |x|, |y| in [2^-500, 2^500]: ratios from 2^-60 to 2^60 (the small-u
    polynomial, the table branches, the pi / 2 and pi folds), equal magnitudes and AP3P-like arguments."""
    rng = np.random.default_rng(8)
    n = 400_000
    y = rng.choice([1, -1], n) * 10.0 ** rng.uniform(-100, 100, n)
    x = y * rng.choice([1, -1], n) * 2.0 ** rng.uniform(-60, 60, n)
    y2 = rng.normal(size=n)
    x2 = rng.normal(size=n)
    t = rng.uniform(0, 1, n)
    y3 = t * rng.choice([1, -1], n)
    x3 = np.ones(n) * rng.choice([1, -1], n)
    s = rng.choice([1.0, -1.0], n // 10)
    A = np.concatenate([y, y2, y3, x3 * s[0], s])
    B = np.concatenate([x, x2, x3, y3, s * rng.choice([1, -1], n // 10)])
    keep = (A != 0) & (B != 0) & (np.abs(A) >= 2.0 ** -500) & (np.abs(A) <= 2.0 ** 500) \
        & (np.abs(B) >= 2.0 ** -500) & (np.abs(B) <= 2.0 ** 500)
    _check(oracle, 8, A[keep], B[keep], name="atan2")
