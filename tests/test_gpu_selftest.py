"""Device self-tests of arithmetic building blocks the parity argument relies on."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_fused_reciprocal_is_correctly_rounded_on_its_domain(native, gpu):
    """rcp_newton (v_rcp_f32 + one FMA Newton step) == IEEE 1.f/w for every 32-bit pattern with
    |w| in [2^-126, 2^126) — the sweep's fast-path domain (exhaustive, 2^32 inputs)."""
    first = np.zeros(16, np.uint32)
    n = native.lib().mcvTestRcpExhaustive(3, first.ctypes.data)
    assert n == 0, [hex(v) for v in first[:min(n, 16)]]


def test_rcp_exact_is_ieee_everywhere(native, gpu):
    """rcp_exact == IEEE 1.f/w for every 32-bit pattern, zeros / denormals / infinities / NaNs
    included — what the certified sweep's exact path (h_error_pk) relies on to reproduce h_error's
    division bit for bit."""
    first = np.zeros(16, np.uint32)
    n = native.lib().mcvTestRcpExhaustive(0, first.ctypes.data)
    assert n == 0, [hex(v) for v in first[:min(n, 16)]]


def test_rcp_exact_bounded_is_ieee_on_its_domain(native, gpu):
    """rcp_exact_bounded (no division branch) == IEEE 1.f/w for every pattern with |w| < 2^126 or NaN."""
    first = np.zeros(16, np.uint32)
    n = native.lib().mcvTestRcpExhaustive(5, first.ctypes.data)
    assert n == 0, [hex(v) for v in first[:min(n, 16)]]


def test_div_fixup_does_not_repair_denormal_reciprocals(native, gpu):
    """v_div_fixup_f32 after rcp_newton handles zeros / infinities / NaNs but not denormal inputs:
    the mismatches of that form are exactly denormal w (why rcp_exact takes the IEEE division there)."""
    first = np.zeros(16, np.uint32)
    n = native.lib().mcvTestRcpExhaustive(2, first.ctypes.data)
    assert n > 0
    for v in first[:16]:
        w = abs(float(np.array([v], np.uint32).view(np.float32)[0]))
        assert w < 2.0**-126 or w >= 2.0**126


def test_reciprocal_mismatches_only_outside_domain(native, gpu):
    """Outside that domain rcp_newton differs from 1.f/w for exactly the 3 * 2^24 patterns with
    |w| < 2^-126 or |w| >= 2^126 (zero/denormal: 2 * 2^23, huge/inf: 2 * 2^23 plus NaNs that
    compare equal): the reason the sweep checks v_cmp_class per point and bounds |w| per hypothesis."""
    first = np.zeros(16, np.uint32)
    n = native.lib().mcvTestRcpExhaustive(1, first.ctypes.data)
    assert n == 3 * 2**24
    for v in first[:16]:
        w = abs(float(np.array([v], np.uint32).view(np.float32)[0]))
        assert w < 2.0**-126 or w >= 2.0**126


def crafted_models():
    """Models whose denominators hit the sweep's rare paths on the test points."""
    rng = np.random.default_rng(0)
    ms = []
    base = np.array([1.02, -0.09, -0.16, 0.08, 1.04, -0.07, 0.40, 0.13], np.float32)
    ms.append(base)
    ms.append(np.array([1, 0, 0, 0, 1, 0, -1, 0], np.float32))          # w = 0 at x = 1
    ms.append(np.array([1, 0, -1, 0, 1, 0, -1, 0], np.float32))         # u = 0 and w = 0 at x = 1
    ms.append(np.array([1, 0, 0, 0, 1, 0, -1.0000001, 0], np.float32))  # tiny w near x = 1
    ms.append(np.array([1, 0, 0, 0, 1, 0, 3e37, 3e37], np.float32))    # huge w -> exact path
    ms.append(np.array([1e-30, 0, 0, 0, 1e-30, 0, 0, 0], np.float32))
    for _ in range(58):
        ms.append((rng.normal(size=8) * rng.choice([1e-3, 1, 10], size=8)).astype(np.float32))
    return np.stack(ms)


@pytest.mark.parametrize("mode", [0, 1, 2, 3])   # op-by-op scalar, fused scalar, fused packed, op-by-op certified
def test_sweep_rare_paths_bit_exact(native, gpu, oracle, mode):
    fused = mode in (1, 2)
    rng = np.random.default_rng(1)
    n = 1000 + 77
    pts = rng.uniform(-1, 1, size=(n, 4)).astype(np.float32)
    pts[:40, 0] = 1.0                       # x = 1: zero denominators for crafted models
    pts[40:60, 0] = np.float32(1.0) / np.float32(1.0000001)
    pts[60:70, :2] = 0.0
    pts[70:80, 2:] = 0.0                    # targets at the origin
    pts[80, 0] = 1e-39                      # denormal coordinate
    models = crafted_models()
    counts = np.zeros(len(models), np.int32)
    thr2 = np.float32(0.05 ** 2)
    ok = native.lib().mcvTestHomographySweep(pts.ctypes.data, n, models.ctypes.data, len(models), float(thr2),
                                             mode, counts.ctypes.data)
    assert ok == 1, native.last_error()
    ref = np.array([oracle.h_count(pts, m, float(thr2), fused=fused) for m in models], np.int32)
    np.testing.assert_array_equal(counts, ref)


def h_err_opcv(pts, h):
    """HomographyEstimatorCallback::computeError op by op in float32 (numpy rounds every operation)."""
    x, y, mx, my = (pts[:, i].astype(np.float32) for i in range(4))
    h = h.astype(np.float32)
    one = np.float32(1)
    with np.errstate(all="ignore"):
        ww = one / (h[6] * x + h[7] * y + one)
        dx = (h[0] * x + h[1] * y + h[2]) * ww - mx
        dy = (h[3] * x + h[4] * y + h[5]) * ww - my
        return dx * dx + dy * dy


def sweep(native, pts, models, thr2, mode):
    counts = np.zeros(len(models), np.int32)
    pts = np.ascontiguousarray(pts, np.float32)
    models = np.ascontiguousarray(models, np.float32)
    ok = native.lib().mcvTestHomographySweep(pts.ctypes.data, pts.shape[0], models.ctypes.data, len(models),
                                             float(thr2), mode, counts.ctypes.data)
    assert ok == 1, native.last_error()
    return counts


@pytest.mark.parametrize("n,scale,seed", [(1077, 1.0, 3), (4096, 1.0, 4), (2049, 640.0, 5), (33, 1.0, 6)])
def test_certified_sweep_at_exact_thresholds(native, gpu, oracle, n, scale, seed):
    """The certified division-free sweep (the default op-by-op path) against the oracle with thresholds
    equal to actual float errors of the points, so that lanes sit exactly on the cut and the exact
    fallback decides them; pixel-scale coordinates included."""
    rng = np.random.default_rng(seed)
    src = rng.uniform(-1, 1, size=(n, 2))
    H = np.array([[1.02, -0.09, -0.16], [0.08, 1.04, -0.07], [0.40, 0.13, 1.0]])
    p = np.c_[src, np.ones(n)] @ H.T
    dst = p[:, :2] / p[:, 2:] + rng.normal(scale=2e-3, size=(n, 2))
    dst[: n // 3] = rng.uniform(-1, 1, size=(n // 3, 2))
    pts = (np.c_[src, dst] * scale).astype(np.float32)
    ms = [H.ravel()[:8] / H[2, 2]]
    for _ in range(31):
        ms.append(ms[0] + rng.normal(scale=1e-3, size=8))
    for _ in range(16):   # random hypotheses, some with the horizon w = 0 crossing the point set
        ms.append(rng.normal(size=8) * np.array([1, 1, 1, 1, 1, 1, 2, 2]))
    models = np.array(ms, np.float64)
    if scale != 1.0:   # same geometry in pixel units: H' = S H S^-1
        models[:, [2, 5]] *= scale
        models[:, [6, 7]] /= scale
    models = models.astype(np.float32)
    for m in models[:4]:
        e = h_err_opcv(pts, m)
        for thr2 in (np.float32(np.median(e)), np.sort(e)[n // 2 + 3], np.float32((5e-3 * scale) ** 2)):
            got = sweep(native, pts, models, thr2, 3)
            ref = np.array([oracle.h_count(pts, mm, float(thr2), fused=False) for mm in models], np.int32)
            np.testing.assert_array_equal(got, ref)
            np.testing.assert_array_equal(ref, [(h_err_opcv(pts, mm) <= thr2).sum() for mm in models])


def test_certified_sweep_near_horizon(native, gpu, oracle):
    """Points on both sides of and right at the line w = 0 of each model (huge projected errors, w of
    either sign, w = +-0 and denormal w): decided by the certified tests or the exact fallback."""
    rng = np.random.default_rng(7)
    n = 3001
    models, pts = [], []
    for _ in range(24):
        h = rng.normal(size=8).astype(np.float32)
        models.append(h)
    models = np.array(models, np.float32)
    x = rng.uniform(-1, 1, size=n).astype(np.float32)
    h = models[0]
    with np.errstate(all="ignore"):
        y = ((-np.float32(1) - h[6] * x) / h[7]).astype(np.float32)   # on the horizon of model 0
    y[::2] = np.nextafter(y[::2], np.float32(np.inf))
    y[::3] = rng.uniform(-1, 1, size=y[::3].shape).astype(np.float32)
    dst = rng.uniform(-50, 50, size=(n, 2)).astype(np.float32)
    pts = np.c_[x, y, dst].astype(np.float32)
    pts = pts[np.isfinite(pts).all(axis=1)]
    for thr2 in (np.float32(1e-2), np.float32(25.0), np.float32(1e6)):
        got = sweep(native, pts, models, thr2, 3)
        ref = np.array([oracle.h_count(pts, m, float(thr2), fused=False) for m in models], np.int32)
        np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("mode", [0, 1, 2, 3])   # random n / reciprocal / exact quotients / domain ends
def test_unscaled_f64_division_matches_ieee(native, gpu, mode):
    """rcp_f64_refined + div_f64_refined (the fp64 division without v_div_scale / v_div_fixup that the
    findScaled and PnP sweeps run) equal the IEEE quotient over 2^26 sampled (n, d) per mode, d in
    +-[2^-64, 2^64]."""
    first = np.zeros(32, np.float64)
    n = native.lib().mcvTestDivF64(mode, 0x5EED + mode, 1 << 26, first.ctypes.data)
    assert n == 0, first[:2 * min(n, 16)].reshape(-1, 2).tolist()


@pytest.mark.parametrize("mode", [4, 5])
def test_unscaled_sqrt_matches_ieee(native, gpu, mode):
    """sqrt_f64_1to2 (the Jacobi rotations' sqrt without the denormal scaling and class select) equals
    the IEEE sqrt over 2^26 sampled x per mode: [1, 2] (the hypots' 1 + r^2, x = 2 included) and
    [0.5, 1] (JacobiSVDImpl_'s cosine / sine arguments, x = 1 included)."""
    first = np.zeros(32, np.float64)
    n = native.lib().mcvTestDivF64(mode, 0x5EED + mode, 1 << 26, first.ctypes.data)
    assert n == 0, first[:2 * min(n, 16)].reshape(-1, 2)[:, 0].tolist()
