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


@pytest.mark.parametrize("mode", [0, 1, 2])   # op-by-op, fused scalar sweep, fused packed sweep
def test_sweep_rare_paths_bit_exact(native, gpu, oracle, mode):
    fused = mode != 0
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


@pytest.mark.parametrize("mode", [0, 1, 2, 3])   # random n / reciprocal / exact quotients / domain ends
def test_unscaled_f64_division_matches_ieee(native, gpu, mode):
    """rcp_f64_refined + div_f64_refined (the fp64 division without v_div_scale / v_div_fixup that the
    findScaled and PnP sweeps run) equal the IEEE quotient over 2^26 sampled (n, d) per mode, d in
    +-[2^-64, 2^64]."""
    first = np.zeros(32, np.float64)
    n = native.lib().mcvTestDivF64(mode, 0x5EED + mode, 1 << 26, first.ctypes.data)
    assert n == 0, first[:2 * min(n, 16)].reshape(-1, 2).tolist()
