"""GPU parity of the PnP path behind cvSolvePnPRansac / cvSolvePnP /
cvRefinePnPLM / cvRefinePnPVVS / solveAp3p (MiniCVNative.cpp:48-163, ap3p.cpp:282-317) against
the oracle (oracle/oracle_pnp.c).
Bar: per-hypothesis poses (AP3P and EPnP kernels), inlier counts and the RANSAC inlier set
bit-exact; the EPnP inlier solve bit-exact in t (the rvec through the host Rodrigues map to 1e-14);
the LM / VVS refined poses within 1e-6 (relative) of the oracle's (GPU sums in another order);
refined poses reach the ground truth on synthetic data."""
import ctypes as C

import numpy as np
import pytest

from minicv_amd import native as N
from minicv_amd import opencv, synthetic as S

pytestmark = pytest.mark.gpu

DIST = [-0.12, 0.03, 0.001, -0.002]


@pytest.fixture(scope="module")
def torch_dev(gpu):
    import torch
    return torch, torch.device("cuda:0")


def rot(r):
    return S.rotation(r / np.linalg.norm(r), np.linalg.norm(r)) if np.linalg.norm(r) > 0 else np.eye(3)


@pytest.mark.parametrize("kind", [5, 1])
@pytest.mark.parametrize("n,outl,seed,begin,count,dist,unfused", [
    (4, 0.0, 1, 0, 32, None, False), (5, 0.2, 2, 0, 100, None, False), (300, 0.5, 3, 0, 256, DIST, False),
    (5000, 0.5, 4, 77777, 100, DIST, False), (2001, 0.6, 5, 0, 300, None, True), (20000, 0.5, 6, 2**31, 64, DIST,
                                                                                  False)])
def test_pnp_counts_bit_exact(torch_dev, oracle, n, outl, seed, begin, count, dist, unfused, kind):
    if kind == 1 and n < 5:
        pytest.skip("EPnP samples 5 points")
    torch, dev = torch_dev
    from minicv_amd import device as D
    img, W, inl, K, d, R, t = S.pnp_problem(n, seed=seed, outlier_frac=outl, dist=dist)
    pts = D.pack_pnp_tensor(img, W, dev)
    pts8 = oracle.pack_pnp(img, W)
    np.testing.assert_array_equal(pts.cpu().numpy(), pts8)
    plan = D.RansacPlan(N.MODEL_PNP, n, count)
    plan.set_camera(K, d)
    thr = 2.0
    cfg = opencv.RansacParams(threshold=thr, seed=seed, fused_error=not unfused).to_c()
    cfg.pnpKind = kind
    key = torch.zeros(2, dtype=torch.int64, device=dev)
    counts = torch.zeros(count, dtype=torch.int32, device=dev)
    plan.evaluate(pts, n, cfg, begin, count, key, counts)
    ref = oracle.pnp_counts(pts8, oracle.cam8(K, d), seed, begin, count, float(np.float32(thr * thr)), not unfused,
                            kind=kind)
    np.testing.assert_array_equal(counts.cpu().numpy(), ref)
    m = 5 if kind == 1 else 4
    if (ref >= m).any() and not (ref == -2).any():
        c = ref.max()
        i = int(np.nonzero(ref == c)[0][0])
        assert int(key[0].item()) == (int(c) << 32) | (0xFFFFFFFF - (begin + i))
    plan.close()


@pytest.mark.parametrize("n,seed,dist,planar", [(1000, 1, DIST, False), (37, 2, None, False), (500, 3, DIST, True),
                                                (6, 4, None, False)])
def test_epnp_hypotheses_bit_exact(native, gpu, oracle, n, seed, dist, planar):
    """The EPnP kernel's poses (one lane per hypothesis, epnp.h) equal the C restatement bit for bit,
    planar targets (zero singular values, cv::RNG branch) and degenerate samples included."""
    img, W, inl, K, d, R, t = S.pnp_problem(n, seed=seed, outlier_frac=0.4, dist=dist)
    if planar:
        W[:, 2] = 0.0
        W[::7] = W[0]                                   # duplicated world points
    pts8 = oracle.pack_pnp(img, W)
    c8 = oracle.cam8(K, d)
    count = 512
    poses = np.zeros((count, 12))
    status = np.zeros(count, np.int32)
    got = native.lib().mcvTestPnpHypotheses(pts8.ctypes.data, n, c8.ctypes.data, 77, 1000, count, 1,
                                            poses.ctypes.data, status.ctypes.data)
    assert got == count, native.last_error()
    for h in range(count):
        st, Ro, to, _ = oracle.pnp_hypothesis_epnp(pts8, c8, 77, 1000 + h)
        assert status[h] == st
        np.testing.assert_array_equal(poses[h, :9], Ro.ravel(), err_msg=f"hyp {h}")
        np.testing.assert_array_equal(poses[h, 9:], to, err_msg=f"hyp {h}")


@pytest.mark.parametrize("fast", [False, True])
def test_ap3p_hypotheses_vs_oracle(native, gpu, oracle, fast):
    """AP3P kernel poses against the oracle, bit for bit. fast (MCV_FLAG_FAST_MINIMAL): the real-root
    finder. Default (the reference's Ferrari quartic + polish, OpenCV's float / pixel input chain): every
    hypothesis is solved on the device with glibc's arithmetic as restated in glibc_math.h — the real-w
    resolvent root through cbrt and csqrt's hypot, the complex-w root (pow(w, 1/3)) through clog's
    log / log1p / hypot, atan2, exp and cos. No hypothesis is handed to the host: every status the kernel
    writes is one of the oracle's (1 ok, -1 no model). Both branch shares are reported; every status and
    every pose equals the glibc oracle."""
    img, W, inl, K, d, R, t = S.pnp_problem(800, seed=5, outlier_frac=0.5, dist=DIST)
    pts8 = oracle.pack_pnp(img, W)
    c8 = oracle.cam8(K, d)
    count = 2048
    poses = np.zeros((count, 12))
    status = np.zeros(count, np.int32)
    kind = 5 | (0x100 if fast else 0)
    assert native.lib().mcvTestPnpHypotheses(pts8.ctypes.data, 800, c8.ctypes.data, 3, 0, count, kind,
                                             poses.ctypes.data, status.ctypes.data) == count
    same = [0, 0]
    finite = [0, 0]
    assert set(np.unique(status)) <= {1, -1}, np.unique(status)
    with oracle.fast_minimal(fast):
        for h in range(count):
            st, Ro, to, _ = oracle.pnp_hypothesis(pts8, c8, 3, h)
            branch = oracle.ap3p_last_branch()
            assert status[h] == st
            if st != 1:
                continue
            ref = np.concatenate([Ro.ravel(), to])
            np.testing.assert_array_equal(poses[h], ref, err_msg=f"hypothesis {h} (branch {branch})")
            if not fast:
                b = max(branch, 0)
                finite[b] += 1
                same[b] += bool(np.array_equal(poses[h], ref))
    if not fast:
        print(f"AP3P Ferrari: real-w (cbrt, on the device) {same[0]} of {finite[0]} poses bit-identical; complex-w "
              f"(glibc's clog / exp / cos / atan2, on the device) {same[1]} of {finite[1]}")
        assert finite[0] > 0 and finite[1] > 0


@pytest.mark.parametrize("kind", [5, 1, 0])
@pytest.mark.parametrize("n,outl,seed,iters,thr,dist,flags", [
    (50, 0.3, 1, 100, 2.0, None, 0), (3000, 0.5, 2, 100, 2.0, DIST, 0), (3000, 0.6, 3, 300, 3.0, None, 0),
    (20000, 0.5, 4, 100, 2.0, DIST, 0), (2000, 0.5, 5, 200, 2.0, None, N.FLAG_FIXED_ITERS | N.FLAG_FUSED_ERROR),
    (2000, 0.5, 6, 200, 2.0, DIST, N.FLAG_NO_REFINE)])
def test_solve_pnp_ransac_vs_oracle(gpu, oracle, n, outl, seed, iters, thr, dist, flags, kind):
    img, W, inl, K, d, R, t = S.pnp_problem(n, seed=seed, outlier_frac=outl, sigma=0.3, dist=dist)
    p = opencv.RansacParams(threshold=thr, confidence=0.99, max_iters=iters, seed=seed,
                            fixed_iters=bool(flags & N.FLAG_FIXED_ITERS), refine=not (flags & N.FLAG_NO_REFINE),
                            fused_error=bool(flags & N.FLAG_FUSED_ERROR))
    name = {0: "Iterative", 1: "EPNP", 5: "AP3P"}[kind]
    ok, r, tt, inliers = opencv.solvePnPRansac(img, W, K, d, kind=name, params=p)
    rc, rr, rt, rmask, best = oracle.solve_pnp_ransac(img, W, K, d, thr=thr, conf=0.99, max_iters=iters, seed=seed,
                                                      flags=flags, kind=kind)
    assert ok and rc > 0
    np.testing.assert_array_equal(inliers, np.nonzero(rmask)[0])
    if flags & N.FLAG_NO_REFINE or kind != 0:
        # the hypothesis pose, or EPnP on the inliers: same bits; rvec via two Rodrigues restatements
        np.testing.assert_allclose(r, rr, rtol=0, atol=1e-14)
        np.testing.assert_array_equal(tt, rt)
    else:
        np.testing.assert_allclose(r, rr, rtol=1e-6, atol=1e-9)
        np.testing.assert_allclose(tt, rt, rtol=1e-6, atol=1e-9)
    if n >= 1000:
        tol = 2e-2 if flags & N.FLAG_NO_REFINE else 2e-3     # unrefined: best minimal-sample pose
        assert np.abs(rot(r) - R).max() < tol and np.abs(tt - t).max() < 10 * tol


@pytest.mark.parametrize("kind", ["EPNP", "Iterative", "DLS"])
def test_five_points_direct_epnp(gpu, oracle, kind):
    """npoints == model_points (5): one EPnP on the float points, all inliers (solvePnPRansac)."""
    img, W, inl, K, d, R, t = S.pnp_problem(5, seed=31, outlier_frac=0, sigma=0, dist=DIST)
    ok, r, tt, inliers = opencv.solvePnPRansac(img, W, K, d, kind=kind, iterations=100, reproj_error=2.0)
    rc, rr, rt, rmask, _ = oracle.solve_pnp_ransac(img, W, K, d, thr=2.0, kind=opencv.SOLVER_KIND[kind])
    assert ok and rc == 5 and list(inliers) == [0, 1, 2, 3, 4]
    np.testing.assert_array_equal(tt, rt)
    np.testing.assert_allclose(r, rr, rtol=0, atol=1e-14)
    assert np.abs(rot(r) - R).max() < 1e-4


def test_solve_pnp_ransac_reference_signature(native, gpu):
    """cvSolvePnPRansac through ctypes exactly like the F# P/Invoke (OpenCV.fs:364-365, :999)."""
    img, W, inl, K, d, R, t = S.pnp_problem(5000, seed=11, outlier_frac=0.5, sigma=0.3)
    for kind in ("Iterative", "EPNP", "P3P", "DLS", "UPNP", "AP3P"):
        ok, r, tt, inliers = opencv.solvePnPRansac(img, W, K, None, kind=kind, iterations=100, reproj_error=2.0,
                                                   confidence=0.99)
        assert ok and len(inliers) > 0.95 * inl.sum() and inl[inliers].mean() > 0.99
        assert np.abs(rot(r) - R).max() < 2e-3


def test_n4_and_solve_pnp(gpu, oracle):
    img, W, inl, K, d, R, t = S.pnp_problem(4, seed=12, outlier_frac=0, sigma=0)
    ok, r, tt, inliers = opencv.solvePnPRansac(img, W, K, None, iterations=100, reproj_error=2.0)
    rc, rr, rt, rmask, _ = oracle.solve_pnp_ransac(img, W, K, None, thr=2.0, flags=N.FLAG_CV_SAMPLER)
    assert ok and list(inliers) == [0, 1, 2, 3] and rc == 4
    np.testing.assert_array_equal(r, rr)
    np.testing.assert_array_equal(tt, rt)
    ok2, r2, t2 = opencv.solvePnP(img, W, K, None, kind="AP3P")
    assert ok2
    np.testing.assert_array_equal(r2, rr)
    with pytest.raises(N.NativeError, match="exactly 4"):
        opencv.solvePnP(np.vstack([img, img[:1]]), np.vstack([W, W[:1]]), K, None, kind="P3P")
    # iterative kind on a clean cloud converges to the truth
    img, W, inl, K, d, R, t = S.pnp_problem(500, seed=13, outlier_frac=0, sigma=0.1, dist=DIST)
    ok3, r3, t3 = opencv.solvePnP(img, W, K, d, kind="Iterative")
    assert ok3 and np.abs(rot(r3) - R).max() < 1e-3 and np.abs(t3 - t).max() < 1e-2
    ok4, r4, t4 = oracle.solve_pnp(img, W, K, d, kind=0)
    np.testing.assert_allclose(r3, r4, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(t3, t4, rtol=1e-6, atol=1e-9)
    # kind 6 (SOLVEPNP_SQPNP): the SQPnP pose, the oracle's to the last bit of t
    ok5, r5, t5 = opencv.solvePnP(img, W, K, d, kind="SQPNP")
    ok6, r6, t6 = oracle.solve_pnp(img, W, K, d, kind=6)
    assert ok5 and ok6
    np.testing.assert_array_equal(t5, t6)
    np.testing.assert_allclose(r5, r6, rtol=0, atol=1e-14)


@pytest.mark.parametrize("n,planar,sigma", [(3, False, 0.0), (4, True, 0.0), (6, False, 0.3), (50, False, 1.0),
                                            (500, True, 0.5), (1024, False, 0.5), (1025, False, 0.5),
                                            (20000, False, 1.0)])
def test_solve_pnp_sqpnp_vs_oracle(gpu, oracle, n, planar, sigma):
    """cvSolvePnP kind 6 (SOLVEPNP_SQPNP, MiniCVNative.cpp:72-74): computeOmega's sums as device passes
    (blocked beyond 1024 points), the SQPnP search on the host; t bit-exact against oracle_sqpnp.c, r
    through the two Rodrigues restatements; noise-free scenes give the pose back."""
    rng = np.random.default_rng(500 + n + planar)
    K = np.array([[800.0, 0, 640], [0, 820.0, 360], [0, 0, 1]])
    R = S.rotation(rng.normal(size=3), rng.uniform(0.0, 1.0))
    t = np.array([rng.normal() * 0.3, rng.normal() * 0.3, rng.uniform(6, 12)])
    W = rng.uniform(-2, 2, size=(n, 3))
    if planar:
        W[:, 2] = 0.0
    Pc = W @ R.T + t
    img = np.c_[Pc[:, 0] / Pc[:, 2] * K[0, 0] + K[0, 2], Pc[:, 1] / Pc[:, 2] * K[1, 1] + K[1, 2]]
    img = img + rng.normal(scale=sigma, size=img.shape)
    d = [-0.05, 0.01, 0.0, 0.001] if n >= 1000 else None
    ok, r, tt = opencv.solvePnP(img, W, K, d, kind="SQPNP")
    ok2, rr, rt = oracle.solve_pnp(img, W, K, d, kind=6)
    assert ok and ok2
    np.testing.assert_array_equal(tt, rt)
    np.testing.assert_allclose(r, rr, rtol=0, atol=1e-14)
    if sigma == 0 and n >= 4:
        assert np.abs(rot(r) - R).max() < 1e-8


def test_solve_pnp_sqpnp_failures(gpu):
    """computeOmega's assertion (coincident image points) and solvePnPGeneric's point count fail with
    the reason; the reference's P/Invoke sees false."""
    K = np.array([[800.0, 0, 640], [0, 820.0, 360], [0, 0, 1]])
    W = np.random.default_rng(0).uniform(-1, 1, size=(10, 3)) + [0, 0, 5]
    with pytest.raises(N.NativeError, match="variance"):
        opencv.solvePnP(np.tile([[600.0, 300.0]], (10, 1)), W, K, None, kind="SQPNP")
    with pytest.raises(N.NativeError, match="at least 3"):
        opencv.solvePnP(np.zeros((2, 2)) + 300.0, W[:2], K, None, kind="SQPNP")


@pytest.mark.parametrize("n,kind", [(6, "EPNP"), (500, "EPNP"), (3000, "UPNP"), (20000, "DLS"), (4, "EPNP")])
def test_solve_pnp_epnp_vs_oracle(gpu, oracle, n, kind):
    """cvSolvePnP with the EPnP family: compute_pose on all double points, bit-exact t (blocked sums
    beyond 1024 points, the device passes against the C restatement)."""
    img, W, inl, K, d, R, t = S.pnp_problem(n, seed=40 + n, outlier_frac=0, sigma=0.2, dist=DIST)
    ok, r, tt = opencv.solvePnP(img, W, K, d, kind=kind)
    ok2, rr, rt = oracle.solve_pnp(img, W, K, d, kind=opencv.SOLVER_KIND[kind])
    assert ok == ok2
    np.testing.assert_array_equal(tt, rt)
    np.testing.assert_allclose(r, rr, rtol=0, atol=1e-14)
    if n >= 500:
        assert np.abs(rot(r) - R).max() < 1e-3


@pytest.mark.parametrize("vvs", [False, True])
def test_refine_converges(gpu, oracle, vvs):
    """cvRefinePnPLM / cvRefinePnPVVS from a perturbed pose: the truth is reached, and the result equals
    the oracle's restatement of the same iteration (sequential sums) to 1e-6 relative."""
    img, W, inl, K, d, R, t = S.pnp_problem(2000, seed=14, outlier_frac=0, sigma=0.05, dist=DIST)
    from minicv_amd.synthetic import rotation
    R0 = rotation([1, 0, 0], 0.05) @ R
    r0 = _rvec(R0)
    t0 = t + np.array([0.05, -0.03, 0.2])
    fn = opencv.refinePnPVVS if vvs else opencv.refinePnPLM
    r, tt = fn(img, W, K, d, r0, t0)
    assert np.abs(rot(r) - R).max() < 1e-3 and np.abs(tt - t).max() < 1e-2
    pts8, c8 = oracle.pack_pnp(img, W), oracle.cam8(K, d)
    rr, rt = oracle.pnp_vvs(pts8, c8, r0, t0) if vvs else oracle.pnp_lm(pts8, c8, r0, t0)
    np.testing.assert_allclose(r, rr, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(tt, rt, rtol=1e-6, atol=1e-9)


def _rvec(R):
    ang = np.arccos(np.clip((np.trace(R) - 1) / 2, -1, 1))
    w = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    return w / (2 * np.sin(ang)) * ang


def test_solve_ap3p_vs_oracle(gpu, oracle):
    """solveAp3p (double arguments, the reference's Ferrari + polish quartic path) against the oracle's
    glibc / std::complex restatement on 1000 random triples: same count and order, every value bit for
    bit (cbrt / hypot restated on the device, the complex-pow branch on the host's glibc)."""
    rng = np.random.default_rng(5)
    K = np.array([[800.0, 0, 640], [0, 820.0, 360], [0, 0, 1]])
    hits = 0
    for c in range(1000):
        R = S.rotation(rng.normal(size=3), rng.uniform(0.0, 1.0))
        t = np.array([rng.normal() * 0.3, rng.normal() * 0.3, rng.uniform(6, 12)])
        W = rng.uniform(-3, 3, size=(3, 3))
        Xc = W @ R.T + t
        img = np.c_[Xc[:, 0] / Xc[:, 2] * K[0, 0] + K[0, 2], Xc[:, 1] / Xc[:, 2] * K[1, 1] + K[1, 2]]
        if c % 3 == 1:
            img = img + rng.normal(scale=20.0, size=img.shape)
        sols = opencv.solveAp3p(img, W, K)
        inv_fx, inv_fy = 1 / K[0, 0], 1 / K[1, 1]
        ref = oracle.solve_ap3p(img[:, 0], img[:, 1], W, inv_fx, inv_fy, K[0, 2] * inv_fx, K[1, 2] * inv_fy)
        assert len(sols) == len(ref), c
        for (Rg, tg), (Ro, to) in zip(sols, ref):
            np.testing.assert_array_equal(Rg, Ro)
            np.testing.assert_array_equal(tg, to)
        if c % 3 != 1:
            hits += min(np.abs(Rg.T - R).max() for Rg, _ in sols) < 1e-6
    assert hits == 667


def test_pnp_edge_cases(gpu):
    K = np.array([[800.0, 0, 640], [0, 820.0, 360], [0, 0, 1]])
    with pytest.raises(N.NativeError, match="at least 4"):
        opencv.solvePnPRansac(np.zeros((3, 2)), np.zeros((3, 3)), K)
    # all world points identical: every AP3P sample is degenerate
    ok, r, t, inl = opencv.solvePnPRansac(np.tile([[600.0, 300.0]], (50, 1)), np.tile([[1.0, 2.0, 3.0]], (50, 1)), K)
    assert not ok and len(inl) == 0
    with pytest.raises(N.NativeError, match="confidence"):
        opencv.solvePnPRansac(*S.pnp_problem(50, seed=1)[:2], K, confidence=1.0)


def _ring_obs(rng, R, t, K, d, W, thr):
    """Observations on / just inside / just outside the threshold circle of pose (R, t)."""
    from test_pnp_cert import _project
    proj = _project(R, t, K, d, W)
    ang = rng.uniform(0, 2 * np.pi, W.shape[0])
    rad = thr * (1 + rng.choice([-1e-6, -1e-7, 0.0, 1e-7, 1e-6, 1e-3], W.shape[0]))
    return proj + np.stack([np.cos(ang), np.sin(ang)], 1) * rad[:, None]


def _sweep(L, pts8, c8, poses, thr2, fused, mode):
    P = np.ascontiguousarray(np.concatenate([np.concatenate([R.ravel(), t]) for R, t in poses]), np.float64)
    counts = np.zeros(len(poses), np.int32)
    r = L.mcvTestPnpSweep(pts8.ctypes.data, pts8.shape[0], c8.ctypes.data, P.ctypes.data, len(poses), thr2,
                          int(fused), int(mode), counts.ctypes.data)
    assert r == len(poses)
    return counts


@pytest.mark.parametrize("n", [1, 2, 127, 128, 129, 1001, 5000])
@pytest.mark.parametrize("fused", [False, True])
def test_pnp_certified_sweep_crafted(native, gpu, oracle, n, fused):
    """The certified packed-fp32 sweep (default) and the all-fp64 sweep on crafted poses — truth,
    perturbed, wild (points behind the camera / on its plane), NaN — over observations crafted onto
    each pose's threshold circle: counts bit-exact against the oracle's exact test per pose."""
    L = native.lib()
    rng = np.random.default_rng(n + 7 * fused)
    img, W, inl, K, d, R, t = S.pnp_problem(n, seed=n, outlier_frac=0.4, sigma=1.0, dist=DIST)
    c8 = oracle.cam8(K, d)
    thr = 2.0
    thr2 = float(np.float32(thr * thr))
    poses = [(R, t)]
    poses += [(S.rotation(rng.normal(size=3), rng.uniform(0, 0.05)) @ R, t + rng.normal(size=3) * 0.05)
              for _ in range(6)]
    poses += [(S.rotation(rng.normal(size=3), rng.uniform(0, np.pi)), rng.normal(size=3) * s) for s in (0.1, 3, 30)]
    poses.append((np.full((3, 3), np.nan), np.zeros(3)))
    poses.append((np.eye(3), np.array([0.0, 0.0, 1e30])))
    for obs in (img, _ring_obs(rng, R, t, K, d, W, thr), _ring_obs(rng, *poses[2], K, d, W, thr)):
        pts8 = oracle.pack_pnp(obs, W)
        ref = np.array([oracle.pnp_count(pts8, c8, Rp, tp, thr2, fused)[0] for Rp, tp in poses])
        for mode in (0, 1):
            np.testing.assert_array_equal(_sweep(L, pts8, c8, poses, thr2, fused, mode), ref)


def test_pnp_certified_sweep_event_overflow(native, gpu, oracle):
    """65536 poses over 30000 points (one point chunk per wave, 235 trips): poses outside the bound's
    domain (non-finite bound) mark every trip undecided, overflow the wave's event list and take the
    exact recount of the chunk; ring observations put undecided lanes into ordinary poses' trips."""
    L = native.lib()
    rng = np.random.default_rng(3)
    n = 30000
    img, W, inl, K, d, R, t = S.pnp_problem(n, seed=11, outlier_frac=0.5, sigma=1.0, dist=DIST)
    c8 = oracle.cam8(K, d)
    thr2 = float(np.float32(4.0))
    obs = img.copy()
    ring = _ring_obs(rng, R, t, K, d, W, 2.0)
    sel = rng.random(n) < 0.02
    obs[sel] = ring[sel]
    pts8 = oracle.pack_pnp(obs, W)
    distinct = [(R, t), (np.eye(3), np.array([0.0, 0.0, 1e30])),
                (S.rotation(rng.normal(size=3), 0.02) @ R, t + 0.02), (np.full((3, 3), np.nan), np.zeros(3))]
    ref = np.array([oracle.pnp_count(pts8, c8, Rp, tp, thr2, False)[0] for Rp, tp in distinct])
    idx = rng.integers(0, len(distinct), 65536)
    counts = _sweep(L, pts8, c8, [distinct[i] for i in idx], thr2, False, 0)
    np.testing.assert_array_equal(counts, ref[idx])


@pytest.mark.slow
@pytest.mark.parametrize("kind", [1, 5])
def test_pnp_counts_bench_workload_full(torch_dev, oracle, kind):
    """bench.py's PnP workload at full size (20k correspondences with k1 k2 p1 p2, 2^20 EPnP / AP3P
    hypotheses in one evaluate): every hypothesis' status / count in a 262144-hypothesis sample over
    the whole range (every 8-rank share's first and last 1024, 240 strided blocks, the bench's
    reported EPnP winner 527,332 and the device's argmax) equals the oracle's."""
    import _sample
    torch, dev = torch_dev
    from minicv_amd import device as D
    n, H = 20_000, 1 << 20
    img, W, inl, K, d, R, t = S.pnp_problem(n, seed=8, outlier_frac=0.5, sigma=0.5, dist=DIST)
    pts = D.pack_pnp_tensor(img, W, dev)
    plan = D.RansacPlan(N.MODEL_PNP, n, H)
    plan.set_camera(K, d)
    cfg = opencv.RansacParams(threshold=2.0, confidence=0.99, max_iters=H, seed=8, fixed_iters=True).to_c()
    cfg.pnpKind = kind
    key = torch.zeros(2, dtype=torch.int64, device=dev)
    counts = torch.zeros(H, dtype=torch.int32, device=dev)
    plan.evaluate(pts, n, cfg, 0, H, key, counts)
    c = counts.cpu().numpy()
    cnt, idx = D.unpack_key(int(key[0].item()))
    assert cnt == c.max() and idx == int(np.argmax(c))
    if kind == 1:
        assert idx == 527_332, "bench.py's reported EPnP winner (profiles/r04_bench_pnp.json)"
    pp8, c8 = oracle.pack_pnp(img, W), oracle.cam8(K, d)
    ranges = _sample.bench_sample(H, around=(idx, 527_332))
    print(f"pnp kind {kind} sample:", _sample.describe(ranges))
    for lo, hi in ranges:
        ref = oracle.pnp_counts(pp8, c8, 8, lo, hi - lo, float(np.float32(4.0)), False, kind=kind)
        np.testing.assert_array_equal(c[lo:hi], ref, err_msg=f"[{lo},{hi})")
    plan.close()
