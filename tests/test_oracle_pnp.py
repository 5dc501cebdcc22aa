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
