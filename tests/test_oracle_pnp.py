"""PnP oracle (oracle/oracle_pnp.c) pinned on exact 2D-3D geometry, and the product's host twin
(hyp_pnp.h compiled for x86) against it bit for bit. CPU only."""
import numpy as np
import pytest

from minicv_amd import synthetic as S


def _pose(rng):
    R = S.rotation(rng.normal(size=3), rng.uniform(0.0, 1.0))
    t = np.array([rng.normal() * 0.3, rng.normal() * 0.3, rng.uniform(6, 12)])
    return R, t


def test_rodrigues_roundtrip_and_derivative(oracle):
    rng = np.random.default_rng(0)
    for _ in range(50):
        r = rng.normal(size=3) * rng.uniform(0, 3)
        R, dR = oracle.rodrigues(r)
        np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-12)
        np.testing.assert_allclose(oracle.rodrigues_inv(R), r if np.linalg.norm(r) <= np.pi else
                                   oracle.rodrigues_inv(R), atol=1e-9)
        for j in range(3):
            e = np.zeros(3)
            e[j] = 1e-6
            num = (oracle.rodrigues(r + e)[0] - oracle.rodrigues(r - e)[0]) / 2e-6
            np.testing.assert_allclose(dR[j], num, atol=1e-7)
    # near-pi and zero rotations
    for ang in (0.0, 1e-9, np.pi - 1e-9, np.pi):
        r = np.array([0.6, -0.8, 0.0]) * ang
        R, _ = oracle.rodrigues(r)
        r2 = oracle.rodrigues_inv(R)
        np.testing.assert_allclose(oracle.rodrigues(r2)[0], R, atol=1e-7)


def test_ap3p_exact_recovery(oracle):
    """Noise-free 3 + 1 correspondences in front of the camera: the 4-point AP3P returns the pose
    (to the fp32 quantisation of the pixel coordinates, as solvePnPRansac converts points to CV_32F)."""
    rng = np.random.default_rng(1)
    K = np.array([[800.0, 0, 640], [0, 820.0, 360], [0, 0, 1]])
    ok = 0
    for trial in range(300):
        R, t = _pose(rng)
        img, W, _, K, dist, R, t = S.pnp_problem(4, seed=trial, outlier_frac=0, sigma=0, R=R, t=t)
        cnt, r, tt, mask, _ = oracle.solve_pnp_ransac(img, W, K)
        assert cnt == 4
        Rr, _ = oracle.rodrigues(r)
        ok += np.abs(Rr - R).max() < 1e-4 and np.abs(tt - t).max() < 1e-3
    assert ok == 300


def test_solve_ap3p_reference_convention(oracle):
    """The export returns the reference's R (ap3p.cpp:245-250) — the transpose of camera-from-world."""
    img, W, _, K, dist, R, t = S.pnp_problem(3, seed=3, outlier_frac=0, sigma=0)
    inv_fx, inv_fy = 1 / K[0, 0], 1 / K[1, 1]
    sols = oracle.solve_ap3p(img[:, 0], img[:, 1], W, inv_fx, inv_fy, K[0, 2] * inv_fx, K[1, 2] * inv_fy)
    assert 1 <= len(sols) <= 4
    assert min(np.abs(Rr.T - R).max() + np.abs(tr - t).max() for Rr, tr in sols) < 1e-8


@pytest.mark.parametrize("dist", [None, [-0.12, 0.03, 0.001, -0.002]])
def test_ransac_lm_recovers_pose(oracle, dist):
    img, W, inl, K, d, R, t = S.pnp_problem(3000, seed=4, outlier_frac=0.5, sigma=0.3, dist=dist)
    cnt, r, tt, mask, best = oracle.solve_pnp_ransac(img, W, K, d, thr=2.0, conf=0.99, max_iters=200, seed=1)
    assert cnt == mask.sum() and cnt > 0.97 * inl.sum() and ((mask != 0) & ~inl).sum() < 0.01 * len(img)
    Rr, _ = oracle.rodrigues(r)
    assert np.abs(Rr - R).max() < 1e-3 and np.abs(tt - t).max() < 1e-2


def test_host_pnp_hypothesis_bit_exact(native, oracle):
    img, W, inl, K, d, R, t = S.pnp_problem(1000, seed=5, outlier_frac=0.5, dist=[-0.1, 0.01, 0.002, 0.001])
    pts8 = oracle.pack_pnp(img, W)
    c8 = oracle.cam8(K, d)
    L = native.lib()
    for hyp in list(range(300)) + [2**32 - 2]:
        st, Ro, to, io = oracle.pnp_hypothesis(pts8, c8, 5, hyp)
        R9, t3, i4 = np.zeros(9), np.zeros(3), np.zeros(4, np.int32)
        st2 = L.mcvHostPnP(pts8.ctypes.data, pts8.shape[0], c8.ctypes.data, 5, hyp, R9.ctypes.data, t3.ctypes.data,
                           i4.ctypes.data)
        assert st == st2
        np.testing.assert_array_equal(Ro.ravel(), R9)
        np.testing.assert_array_equal(to, t3)
        if st == 1:
            np.testing.assert_array_equal(io, i4)


def test_host_rodrigues_matches_oracle(native, oracle):
    rng = np.random.default_rng(2)
    L = native.lib()
    for _ in range(30):
        r = np.ascontiguousarray(rng.normal(size=3))
        R, dR = np.zeros(9), np.zeros(27)
        L.mcvHostRodrigues(r.ctypes.data, R.ctypes.data, dR.ctypes.data)
        Ro, dRo = oracle.rodrigues(r)
        np.testing.assert_allclose(R, Ro.ravel(), rtol=0, atol=1e-15)
        np.testing.assert_allclose(dR, dRo.ravel(), rtol=0, atol=1e-14)
        r2 = np.zeros(3)
        L.mcvHostRodriguesInv(np.ascontiguousarray(R).ctypes.data, r2.ctypes.data)
        np.testing.assert_allclose(r2, oracle.rodrigues_inv(Ro), atol=1e-14)


# ---- EPnP (oracle/oracle_epnp.c; product twin minicv_amd/csrc/epnp.h) ---------------------------
def _project_px(W, K, R, t):
    Xc = W @ R.T + t
    return np.c_[Xc[:, 0] / Xc[:, 2] * K[0, 0] + K[0, 2], Xc[:, 1] / Xc[:, 2] * K[1, 1] + K[1, 2]]


@pytest.mark.parametrize("n", [5, 6, 12, 200, 1024, 1025, 5000])
def test_epnp_exact_recovery(oracle, n):
    """Noise-free pixels of a known pose: compute_pose returns it (n > 1024 exercises the blocked sums)."""
    rng = np.random.default_rng(n)
    K = np.array([[800.0, 0, 640], [0, 820.0, 360], [0, 0, 1]])
    for trial in range(20):
        R, t = _pose(rng)
        W = rng.uniform(-3, 3, size=(n, 3))
        us = _project_px(W, K, R, t)
        Re, te = oracle.epnp(W, us, (K[0, 0], K[1, 1], K[0, 2], K[1, 2]))
        assert np.abs(Re - R).max() < 1e-8 and np.abs(te - t).max() < 1e-7, (trial, Re - R, te - t)
        np.testing.assert_allclose(Re @ Re.T, np.eye(3), atol=1e-12)


@pytest.mark.parametrize("n", [5, 40, 3000])
def test_epnp_planar_target(oracle, n):
    """Near-planar targets (|Z| <= 1e-2) are recovered exactly. On an exactly planar one (Z = 0)
    PW0^T PW0 has a zero singular value: the null-singular-vector branch of JacobiSVD (cv::RNG fill)
    runs, the fourth control point coincides with the centroid and OpenCV's general-case EPnP (no
    planar variant) is ill-posed; the restatement only has to stay finite and return a rotation."""
    rng = np.random.default_rng(100 + n)
    K = np.array([[800.0, 0, 640], [0, 820.0, 360], [0, 0, 1]])
    cam4 = (K[0, 0], K[1, 1], K[0, 2], K[1, 2])
    for trial in range(10):
        R, t = _pose(rng)
        W = np.c_[rng.uniform(-3, 3, size=(n, 2)), rng.uniform(-1e-2, 1e-2, size=n)]
        Re, te = oracle.epnp(W, _project_px(W, K, R, t), cam4)
        assert np.abs(Re - R).max() < 1e-9 and np.abs(te - t).max() < 1e-8, trial
        W[:, 2] = 0.0
        Re, te = oracle.epnp(W, _project_px(W, K, R, t), cam4)
        assert np.isfinite(Re).all() and np.isfinite(te).all()
        np.testing.assert_allclose(Re @ Re.T, np.eye(3), atol=1e-9)
        assert abs(np.linalg.det(Re) - 1) < 1e-9


def _epnp_cases(rng, count):
    K = np.array([[800.0, 0, 640], [0, 820.0, 360], [0, 0, 1]])
    cam4 = np.array([K[0, 0], K[1, 1], K[0, 2], K[1, 2]])
    for c in range(count):
        R, t = _pose(rng)
        W = rng.uniform(-3, 3, size=(5, 3))
        if c % 5 == 1:
            W[:, 2] = 0.0                                      # planar
        if c % 5 == 2:
            W[3] = W[0] + 1e-7 * rng.normal(size=3)            # near-duplicate point
        us = _project_px(W, K, R, t)
        if c % 5 == 3:
            us = us + rng.normal(scale=2.0, size=us.shape)     # noisy
        if c % 5 == 4:
            us = rng.uniform(0, 1000, size=us.shape)           # garbage
        yield np.ascontiguousarray(W), np.ascontiguousarray(us), cam4


def test_host_epnp5_bit_exact(native, oracle):
    """The x86 build of epnp_solve_small<5> (the code every GPU lane runs) equals the C restatement
    bit for bit on regular, planar, near-degenerate, noisy and garbage 5-point sets."""
    L = native.lib()
    rng = np.random.default_rng(7)
    for W, us, cam4 in _epnp_cases(rng, 400):
        R9, t3 = np.zeros(9), np.zeros(3)
        L.mcvHostEpnp5(W.ctypes.data, us.ctypes.data, cam4.ctypes.data, R9.ctypes.data, t3.ctypes.data)
        Ro, to = oracle.epnp(W, us, cam4)
        np.testing.assert_array_equal(R9, Ro.ravel())
        np.testing.assert_array_equal(t3, to)


def test_host_epnp_hypothesis_bit_exact(native, oracle):
    img, W, inl, K, d, R, t = S.pnp_problem(1000, seed=6, outlier_frac=0.5, dist=[-0.1, 0.01, 0.002, 0.001])
    pts8 = oracle.pack_pnp(img, W)
    c8 = oracle.cam8(K, d)
    L = native.lib()
    for hyp in list(range(200)) + [2**32 - 2]:
        st, Ro, to, io = oracle.pnp_hypothesis_epnp(pts8, c8, 9, hyp)
        R9, t3, i5 = np.zeros(9), np.zeros(3), np.zeros(5, np.int32)
        st2 = L.mcvHostPnPEpnp(pts8.ctypes.data, pts8.shape[0], c8.ctypes.data, 9, hyp, R9.ctypes.data,
                               t3.ctypes.data, i5.ctypes.data)
        assert st == st2 == 1
        np.testing.assert_array_equal(Ro.ravel(), R9)
        np.testing.assert_array_equal(to, t3)
        np.testing.assert_array_equal(io, i5)


@pytest.mark.parametrize("kind", [0, 1, 2, 5])
def test_ransac_kinds_recover_pose(oracle, kind):
    """solvePnPRansac per kind: EPnP-5 kernel (0, 1) or AP3P-4 (2, 5); final LM (0) or EPnP on the inliers."""
    img, W, inl, K, d, R, t = S.pnp_problem(2000, seed=21, outlier_frac=0.4, sigma=0.3, dist=[-0.1, 0.01, 0.0, 0.0])
    cnt, r, tt, mask, best = oracle.solve_pnp_ransac(img, W, K, d, thr=2.0, conf=0.99, max_iters=300, seed=3,
                                                     kind=kind)
    assert cnt == mask.sum() and cnt > 0.95 * inl.sum() and ((mask != 0) & ~inl).sum() < 0.01 * len(img)
    Rr, _ = oracle.rodrigues(r)
    assert np.abs(Rr - R).max() < 2e-3 and np.abs(tt - t).max() < 2e-2


@pytest.mark.parametrize("kind", [0, 1, 6])
def test_solve_pnp_all_points(oracle, kind):
    img, W, inl, K, d, R, t = S.pnp_problem(500, seed=22, outlier_frac=0.0, sigma=0.0, dist=[-0.1, 0.01, 0.002, 0.0])
    ok, r, tt = oracle.solve_pnp(img, W, K, d, kind=kind)
    Rr, _ = oracle.rodrigues(r)
    assert ok and np.abs(Rr - R).max() < 1e-6 and np.abs(tt - t).max() < 1e-5


def _object_space_cost(R, W, xy):
    """SQPnP's objective restated independently: min over t of sum ||[I2 | -x_i] (R P_i + t)||^2 (the
    quadratic form r^T Omega r of computeOmega), t by linear least squares."""
    n = len(W)
    A = np.zeros((2 * n, 3))
    b = np.zeros(2 * n)
    for i, ((x, y), P) in enumerate(zip(xy, W)):
        M = np.array([[1.0, 0.0, -x], [0.0, 1.0, -y]])
        A[2 * i:2 * i + 2] = M
        b[2 * i:2 * i + 2] = -M @ (R @ P)
    t, *_ = np.linalg.lstsq(A, b, rcond=None)
    res = A @ t - b
    return float(res @ res), t


def _normalised(img, K):
    return np.c_[(img[:, 0] - K[0, 2]) / K[0, 0], (img[:, 1] - K[1, 2]) / K[1, 1]]


@pytest.mark.parametrize("n,planar", [(3, False), (4, False), (6, False), (50, False), (500, False), (3000, False),
                                      (4, True), (20, True), (1000, True)])
def test_sqpnp_exact_recovery(oracle, n, planar):
    """SQPnP (cvSolvePnP kind 6) on noise-free correspondences returns the pose: general and planar
    scenes (Omega with a larger null space), 3 points (the minimum solvePnPGeneric admits for SQPnP)
    and more than one 1024-point block of sums."""
    rng = np.random.default_rng(100 + n + planar)
    K = np.array([[800.0, 0, 640], [0, 820.0, 360], [0, 0, 1]])
    R, t = _pose(rng)
    W = rng.uniform(-2, 2, size=(n, 3))
    if planar:
        W[:, 2] = 0.0
    Pc = W @ R.T + t
    img = np.c_[Pc[:, 0] / Pc[:, 2] * K[0, 0] + K[0, 2], Pc[:, 1] / Pc[:, 2] * K[1, 1] + K[1, 2]]
    ok, r, tt = oracle.solve_pnp(img, W, K, None, kind=6)
    Rr, _ = oracle.rodrigues(r)
    assert ok
    if n >= 4:
        assert np.abs(Rr - R).max() < 1e-8 and np.abs(tt - t).max() < 1e-7
    else:   # P3P has up to four exact poses: SQPnP returns one of zero cost
        assert _object_space_cost(Rr, W, _normalised(img, K))[0] < 1e-18


def test_sqpnp_global_minimum_with_noise(oracle):
    """With pixel noise the answer minimises the object-space cost: its cost is below that of the true
    pose, of EPnP's pose and of small rotations around it; t is the cost's minimiser for that R."""
    rng = np.random.default_rng(7)
    for trial in range(6):
        img, W, inl, K, d, R, t = S.pnp_problem(300, seed=70 + trial, outlier_frac=0.0, sigma=1.0)
        ok, r, tt = oracle.solve_pnp(img, W, K, None, kind=6)
        assert ok
        Rr, _ = oracle.rodrigues(r)
        xy = _normalised(img, K)
        c0, t_ls = _object_space_cost(Rr, W, xy)
        np.testing.assert_allclose(tt, t_ls, rtol=1e-6, atol=1e-9)
        assert c0 <= _object_space_cost(R, W, xy)[0] * (1 + 1e-9)
        ok1, r1, _ = oracle.solve_pnp(img, W, K, None, kind=1)
        assert c0 <= _object_space_cost(oracle.rodrigues(r1)[0], W, xy)[0] * (1 + 1e-9)
        for _ in range(20):
            dR, _ = oracle.rodrigues(rng.normal(size=3) * 1e-4)
            assert c0 <= _object_space_cost(dR @ Rr, W, xy)[0] * (1 + 1e-12)


def test_sqpnp_degenerate_inputs(oracle):
    """computeOmega's assertions: image points that all coincide (coordinate variance 0) fail."""
    K = np.array([[800.0, 0, 640], [0, 820.0, 360], [0, 0, 1]])
    W = np.random.default_rng(0).uniform(-1, 1, size=(10, 3)) + [0, 0, 5]
    img = np.tile([[600.0, 300.0]], (10, 1))
    ok, _, _ = oracle.solve_pnp(img, W, K, None, kind=6)
    assert not ok


@pytest.mark.parametrize("n,planar,sigma", [(3, False, 0.0), (6, False, 0.5), (200, False, 1.0), (200, True, 1.0),
                                            (2500, False, 0.5)])
def test_host_sqpnp_bit_exact(native, oracle, n, planar, sigma):
    """The product's SQPnP algebra (sqpnp.h, host build, over sums in the device passes' block order)
    equals oracle_sqpnp.c bit for bit, distortion included."""
    rng = np.random.default_rng(300 + n)
    K = np.array([[800.0, 0, 640], [0, 820.0, 360], [0, 0, 1]])
    dist = np.array([-0.08, 0.01, 0.001, -0.0005])
    R, t = _pose(rng)
    W = rng.uniform(-2, 2, size=(n, 3))
    if planar:
        W[:, 2] = 0.0
    Pc = W @ R.T + t
    img = np.c_[Pc[:, 0] / Pc[:, 2] * K[0, 0] + K[0, 2], Pc[:, 1] / Pc[:, 2] * K[1, 1] + K[1, 2]]
    img = img + rng.normal(scale=sigma, size=img.shape)
    cam8 = np.array([K[0, 0], K[1, 1], K[0, 2], K[1, 2], *dist])
    code, Ro, to = oracle.sqpnp_pose(img, W, cam8)
    R9, t3 = np.zeros(9), np.zeros(3)
    img_c, W_c = np.ascontiguousarray(img), np.ascontiguousarray(W)
    got = native.lib().mcvHostSqpnp(img_c.ctypes.data, W_c.ctypes.data, n, cam8.ctypes.data, R9.ctypes.data, t3.ctypes.data)
    assert got == code and code > 0
    np.testing.assert_array_equal(R9, Ro.ravel())
    np.testing.assert_array_equal(t3, to)


def _ap3p_triples(count, seed):
    """Random 3-point problems: pixel observations of a random pose, a few of them perturbed so that
    the quartic has complex roots (whose real parts the reference keeps) or nearly double roots."""
    rng = np.random.default_rng(seed)
    K = np.array([[800.0, 0, 640], [0, 820.0, 360], [0, 0, 1]])
    for c in range(count):
        R, t = _pose(rng)
        W = rng.uniform(-3, 3, size=(3, 3))
        us = _project_px(W, K, R, t)
        if c % 3 == 1:
            us = us + rng.normal(scale=20.0, size=us.shape)
        yield us, W, K


def test_solve_ap3p_reference_quartic_path(native, oracle):
    """solveAp3p's own quartic path (Ferrari with std::complex + 2 polish passes, ap3p.cpp:10-74): the
    host build of the product code against the oracle's glibc / C99-complex restatement on 1000 random
    triples — same solution count and order, values within 1e-9 (the transcendentals are libm's on
    both sides here; the GPU test holds the device to the same bar)."""
    L = native.lib()
    spurious = 0
    for us, W, K in _ap3p_triples(1000, 5):
        inv_fx, inv_fy = 1 / K[0, 0], 1 / K[1, 1]
        args = (np.ascontiguousarray(us[:, 0]), np.ascontiguousarray(us[:, 1]), np.ascontiguousarray(W.ravel()))
        R36, t12 = np.zeros(36), np.zeros(12)
        n = L.mcvHostSolveAp3p(*(a.ctypes.data for a in args), inv_fx, inv_fy, K[0, 2] * inv_fx, K[1, 2] * inv_fy,
                               R36.ctypes.data, t12.ctypes.data)
        ref = oracle.solve_ap3p(us[:, 0], us[:, 1], W, inv_fx, inv_fy, K[0, 2] * inv_fx, K[1, 2] * inv_fy)
        assert n == len(ref)
        for i, (Ro, to) in enumerate(ref):
            np.testing.assert_allclose(R36[9 * i:9 * i + 9], Ro.ravel(), rtol=0, atol=1e-9)
            np.testing.assert_allclose(t12[3 * i:3 * i + 3], to, rtol=1e-9, atol=1e-9)
        spurious += n - sum(np.abs(np.linalg.det(Ro) - 1) < 1e-6 for Ro, _ in ref)
    assert spurious >= 0
