"""Certified packed-fp32 PnP prefilter (minicv_amd/csrc/pnp_pk.h) through its host twin: every lane
it decides must equal the exact fp64 test (hyp_pnp.h pnp_error, the reference's
PnPRansacCallback::computeError restated), on true, perturbed and wild poses, with distortion, with
points crafted onto the threshold circle, behind the camera and on its plane. CPU only (the GPU
sweep's counts are checked against the oracle in test_gpu_pnp.py)."""
import numpy as np
import pytest

from minicv_amd import synthetic as S

DISTS = [None, [0.08, -0.02, 0.001, -0.0015], [-0.3, 0.12, 0.004, 0.003]]


def _cert(L, pts8, c8, R, t, thr2, fused):
    n = pts8.shape[0]
    dec = np.zeros(n, np.int32)
    ex = np.zeros(n, np.int32)
    R9 = np.ascontiguousarray(R, np.float64).ravel()
    t3 = np.ascontiguousarray(t, np.float64)
    bad = L.mcvHostPnpCert(pts8.ctypes.data, n, c8.ctypes.data, R9.ctypes.data, t3.ctypes.data, thr2, int(fused),
                           dec.ctypes.data, ex.ctypes.data)
    return bad, dec, ex


def _project(R, t, K, d, W):
    Xc = W @ R.T + t
    x, y = Xc[:, 0] / Xc[:, 2], Xc[:, 1] / Xc[:, 2]
    r2 = x * x + y * y
    cd = 1 + d[0] * r2 + d[1] * r2 * r2
    xd = x * cd + d[2] * 2 * x * y + d[3] * (r2 + 2 * x * x)
    yd = y * cd + d[2] * (r2 + 2 * y * y) + d[3] * 2 * x * y
    return np.stack([xd * K[0, 0] + K[0, 2], yd * K[1, 1] + K[1, 2]], axis=1)


@pytest.mark.parametrize("di", range(len(DISTS)))
@pytest.mark.parametrize("fused", [False, True])
def test_cert_decisions_equal_exact(native, oracle, di, fused):
    L = native.lib()
    dist = DISTS[di]
    img, W, inl, K, d, R, t = S.pnp_problem(4000, seed=21 + di, outlier_frac=0.5, sigma=1.0, dist=dist)
    c8 = oracle.cam8(K, d)
    rng = np.random.default_rng(100 + di)
    thr = 2.0
    total = und = 0
    poses = [(R, t)]
    for _ in range(12):   # perturbed poses (the RANSAC hypotheses near the truth)
        poses.append((S.rotation(rng.normal(size=3), rng.uniform(0, 0.05)) @ R, t + rng.normal(size=3) * 0.05))
    for _ in range(12):   # wild poses: points behind the camera, on its plane, far off-image
        Rw = S.rotation(rng.normal(size=3), rng.uniform(0, np.pi))
        tw = rng.normal(size=3) * rng.choice([0.1, 3.0, 30.0])
        poses.append((Rw, tw))
    for Rp, tp in poses:
        # observations on / just inside / just outside the threshold circle of this pose
        proj = _project(Rp, tp, K, d, W)
        ang = rng.uniform(0, 2 * np.pi, W.shape[0])
        rad = thr * (1 + rng.choice([-1e-6, -1e-7, 0.0, 1e-7, 1e-6, 1e-3], W.shape[0]))
        ring = proj + np.stack([np.cos(ang), np.sin(ang)], 1) * rad[:, None]
        for obs in (img, ring):
            pts8 = oracle.pack_pnp(obs, W)
            bad, dec, ex = _cert(L, pts8, c8, Rp, tp, np.float32(thr * thr), fused)
            assert bad == 0, f"{bad} decided lanes differ from the exact test"
            badc, decc, _ = _cert(L, pts8, c8, Rp, tp, np.float32(thr * thr), int(fused) | 2)
            assert badc == 0, f"cheap tier: {badc} decided lanes differ from the exact test"
            assert ((decc < 0) | (decc == dec)).all()
            m = np.isfinite(obs).all(axis=1)
            total += int(m.sum())
            und += int((dec[m] < 0).sum())
    # the true pose on the benchmark-like data: essentially everything decided, nearly all of it by the
    # cheap tier
    pts8 = oracle.pack_pnp(img, W)
    _, dec, _ = _cert(L, pts8, c8, R, t, np.float32(thr * thr), fused)
    assert (dec < 0).mean() < 1e-3
    _, decc, _ = _cert(L, pts8, c8, R, t, np.float32(thr * thr), int(fused) | 2)
    assert (decc < 0).mean() < 0.02


def test_cert_edge_inputs(native, oracle):
    """Non-finite points, zero threshold, points exactly on the camera plane (Zc == 0: the exact path
    divides by 1), huge coordinates: decided lanes still equal the exact test."""
    L = native.lib()
    img, W, inl, K, d, R, t = S.pnp_problem(512, seed=5, outlier_frac=0.3, sigma=0.5, dist=DISTS[1])
    c8 = oracle.cam8(K, d)
    W = W.copy()
    img = img.copy()
    W[0] = [np.nan, 0, 0]
    W[1] = [np.inf, 1, 1]
    img[2] = [np.nan, 5]
    # points on the camera plane: Zc = R[2] . X + t2 = 0
    for i in range(3, 8):
        X = W[i].copy()
        X[2] = -(R[2, 0] * X[0] + R[2, 1] * X[1] + t[2]) / R[2, 2]
        W[i] = X
    W[8] = [1e20, -1e20, 1e20]
    for thr2 in (np.float32(0.0), np.float32(1e-12), np.float32(4.0), np.float32(1e12)):
        for fused in (False, True):
            pts8 = oracle.pack_pnp(img, W)
            bad, dec, ex = _cert(L, pts8, c8, R, t, thr2, fused)
            assert bad == 0
            assert _cert(L, pts8, c8, R, t, thr2, int(fused) | 2)[0] == 0
    # a non-finite extent disables certification for every lane (all undecided)
    pts8 = oracle.pack_pnp(img, W)
    _, dec, _ = _cert(L, pts8, c8, R, t, np.float32(4.0), False)
    assert (dec < 0).all()
