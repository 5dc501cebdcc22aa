"""Seeded synthetic workloads for the BASELINE.json configs (no datasets: no network).

Shapes follow SURVEY.md §8d / BASELINE.md §2:
  cfg1/cfg3  homography: src ~ U[-1,1]^2 (NDC convention, OpenCV.fs:873-876), dst = pi(H_true src)
             with H_true = the matrix of the reference's cvTest export (MiniCVNative.cpp:506-511,
             as cvTest builds it), inliers + N(0, sigma), a fraction of outliers ~ U[-1,1]^2
             (50 % as in the authors' synthetic test, Program.fs:10-12), thr 5e-3 (OpenCV.fs:34).
  cfg2       Hamming: train bits ~ Bernoulli(0.5); queries = planted train rows with 0-40 flipped
             bits, 10 % pure random queries.
  cfg4       fundamental: two lookAt cameras (src/Test/Camera.fs:171-184 model) viewing points in
             a 6-unit cube (Program.fs:14), projections + N(0, sigma), 50 % outliers.
  cfg5       SIFT-like fp32 descriptors: |N(0,1)| -> L2-normalise -> x512 -> clip 255, planted
             near-duplicates.
"""
from __future__ import annotations

import numpy as np

# cvTest (MiniCVNative.cpp:506-511): arr1 is transposed into arr, and H = Mat(3,3,arr).
_ARR1 = np.array([1.02736340896169, 0.0824668492092278, 0.399551267404442, -0.0921929548453944,
                  1.03823834690651, 0.12968385038247, -0.159700861517284, -0.0688464520524622, 1.0])
H_TRUE = _ARR1.reshape(3, 3).T.copy()


def project(H: np.ndarray, p: np.ndarray) -> np.ndarray:
    x = p @ H[:, :2].T + H[:, 2]
    return x[:, :2] / x[:, 2:3]


def homography_problem(n: int, seed: int, outlier_frac: float = 0.5, sigma: float = 1e-3, H: np.ndarray = H_TRUE):
    """-> src (n,2) f64, dst (n,2) f64, is_inlier (n,) bool"""
    rng = np.random.default_rng(seed)
    src = rng.uniform(-1, 1, size=(n, 2))
    dst = project(H, src) + rng.normal(0, sigma, size=(n, 2))
    out = rng.random(n) < outlier_frac
    dst[out] = rng.uniform(-1, 1, size=(int(out.sum()), 2))
    return src, dst, ~out


def hamming_problem(nq: int, nt: int, nbytes: int = 32, seed: int = 2, random_frac: float = 0.1,
                    max_flips: int = 40):
    """-> q (nq, nbytes) u8, t (nt, nbytes) u8, planted (nq,) int (-1 for random queries)"""
    rng = np.random.default_rng(seed)
    t = rng.integers(0, 256, size=(nt, nbytes), dtype=np.uint8)
    planted = rng.integers(0, nt, size=nq)
    q = t[planted].copy()
    bits = np.unpackbits(q, axis=1)
    flips = rng.integers(0, min(max_flips, nbytes * 8) + 1, size=nq)
    for i in range(nq):
        pos = rng.choice(nbytes * 8, size=flips[i], replace=False)
        bits[i, pos] ^= 1
    q = np.packbits(bits, axis=1)
    rnd = rng.random(nq) < random_frac
    q[rnd] = rng.integers(0, 256, size=(int(rnd.sum()), nbytes), dtype=np.uint8)
    planted[rnd] = -1
    return q, t, planted


def sift_like(n: int, dim: int, rng) -> np.ndarray:
    d = np.abs(rng.normal(size=(n, dim)))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return np.minimum(d * 512.0, 255.0).astype(np.float32)


def l2_problem(nq: int, nt: int, dim: int = 128, seed: int = 5, noise: float = 2.0, random_frac: float = 0.1):
    rng = np.random.default_rng(seed)
    t = sift_like(nt, dim, rng)
    planted = rng.integers(0, nt, size=nq)
    q = np.clip(t[planted] + rng.normal(0, noise, size=(nq, dim)), 0, 255).astype(np.float32)
    rnd = rng.random(nq) < random_frac
    q[rnd] = sift_like(int(rnd.sum()), dim, rng)
    planted[rnd] = -1
    return q, t, planted


def look_at(eye, target, up):
    """World->camera rotation/translation of a lookAt camera (camera looks down -z)."""
    eye, target, up = map(lambda v: np.asarray(v, dtype=np.float64), (eye, target, up))
    f = target - eye
    f /= np.linalg.norm(f)
    r = np.cross(f, up)
    r /= np.linalg.norm(r)
    u = np.cross(r, f)
    R = np.stack([r, u, -f])
    return R, -R @ eye


def fundamental_problem(n: int, seed: int = 4, outlier_frac: float = 0.5, sigma: float = 1e-3):
    """Two pinhole cameras (identity intrinsics, NDC image plane) viewing points in a 6-unit cube.
    -> a (n,2), b (n,2), is_inlier, F_true (3x3, b^T F a = 0)"""
    rng = np.random.default_rng(seed)
    X = rng.uniform(-3, 3, size=(n, 3))
    R1, t1 = look_at([4.0, 5.0, 6.0], [0, 0, 0], [0, 0, 1])
    R2, t2 = look_at([6.0, -3.0, 5.0], [0, 0, 0], [0, 0, 1])

    def proj(R, t):
        c = X @ R.T + t
        return -c[:, :2] / c[:, 2:3]   # camera looks down -z; image coords (x, y) / depth

    a = proj(R1, t1) + rng.normal(0, sigma, size=(n, 2))
    b = proj(R2, t2) + rng.normal(0, sigma, size=(n, 2))
    out = rng.random(n) < outlier_frac
    lo, hi = b.min(axis=0), b.max(axis=0)
    b[out] = rng.uniform(lo, hi, size=(int(out.sum()), 2))
    # F from relative pose: x2 ~ K(R x1 + t); with the -z convention the image point is (-X/Z, -Y/Z)
    R = R2 @ R1.T
    t = t2 - R @ t1
    tx = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])
    E = tx @ R
    S = np.diag([1.0, 1.0, -1.0])   # image (x, y, 1) = S * normalised camera ray up to scale
    F = S @ E @ S
    return a, b, ~out, F / np.linalg.norm(F)


def rotation(axis, angle_rad: float) -> np.ndarray:
    """Rodrigues rotation matrix."""
    k = np.asarray(axis, dtype=np.float64)
    k = k / np.linalg.norm(k)
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(angle_rad) * K + (1 - np.cos(angle_rad)) * K @ K


def essential_problem(n: int, seed: int = 6, outlier_frac: float = 0.5, sigma: float = 0.3, focal: float = 800.0,
                      pp=(640.0, 360.0), R: np.ndarray | None = None, t=None):
    """Calibrated two-view pixels (OpenCV convention: camera looks down +z, x = f X/Z + pp).
    Camera 1 = [I | 0]; camera 2 = [R | t] (X2 = R X1 + t). Points at depth 4..12.
    -> a (n,2), b (n,2), is_inlier, R, t_unit, E_true (unit norm, x2n^T E x1n = 0)"""
    rng = np.random.default_rng(seed)
    R = rotation([0.2, 1.0, 0.1], np.deg2rad(8.0)) if R is None else np.asarray(R, dtype=np.float64)
    t = np.array([1.0, 0.15, 0.1]) if t is None else np.asarray(t, dtype=np.float64)
    X = np.stack([rng.uniform(-3, 3, n), rng.uniform(-2, 2, n), rng.uniform(4, 12, n)], axis=1)
    Y = X @ R.T + t
    ppa = np.asarray(pp, dtype=np.float64)
    a = focal * X[:, :2] / X[:, 2:3] + ppa + rng.normal(0, sigma, size=(n, 2))
    b = focal * Y[:, :2] / Y[:, 2:3] + ppa + rng.normal(0, sigma, size=(n, 2))
    out = rng.random(n) < outlier_frac
    lo, hi = b.min(axis=0), b.max(axis=0)
    b[out] = rng.uniform(lo, hi, size=(int(out.sum()), 2))
    tu = t / np.linalg.norm(t)
    tx = np.array([[0, -tu[2], tu[1]], [tu[2], 0, -tu[0]], [-tu[1], tu[0], 0]])
    E = tx @ R
    return a, b, ~out, R, tu, E / np.linalg.norm(E)


def pnp_problem(n: int, seed: int = 8, outlier_frac: float = 0.5, sigma: float = 0.5, K=None, dist=None,
                R: np.ndarray | None = None, t=None):
    """2D-3D correspondences (OpenCV camera: x = K (R X + t), +z forward) after the reference's
    testPnp recipe (Program.fs:8-24: points in a 6-unit cube). Optional distortion (k1, k2, p1, p2)
    is applied with the projectPoints model. -> img (n,2), world (n,3), is_inlier, K, dist, R, t"""
    rng = np.random.default_rng(seed)
    K = np.array([[800.0, 0, 640.0], [0, 820.0, 360.0], [0, 0, 1]]) if K is None else np.asarray(K, np.float64)
    dist = np.zeros(4) if dist is None else np.asarray(dist, np.float64)
    R = rotation([0.3, -1.0, 0.2], np.deg2rad(25.0)) if R is None else np.asarray(R, np.float64)
    t = np.array([0.2, -0.1, 9.0]) if t is None else np.asarray(t, np.float64)
    W = rng.uniform(-3, 3, size=(n, 3))
    Xc = W @ R.T + t
    x, y = Xc[:, 0] / Xc[:, 2], Xc[:, 1] / Xc[:, 2]
    r2 = x * x + y * y
    cd = 1 + dist[0] * r2 + dist[1] * r2 * r2
    xd = x * cd + dist[2] * 2 * x * y + dist[3] * (r2 + 2 * x * x)
    yd = y * cd + dist[2] * (r2 + 2 * y * y) + dist[3] * 2 * x * y
    img = np.stack([xd * K[0, 0] + K[0, 2], yd * K[1, 1] + K[1, 2]], axis=1) + rng.normal(0, sigma, size=(n, 2))
    out = rng.random(n) < outlier_frac
    lo, hi = img.min(axis=0), img.max(axis=0)
    img[out] = rng.uniform(lo, hi, size=(int(out.sum()), 2))
    return img, W, ~out, K, dist, R, t


H_PIX = np.array([[1.05, 0.02, 15.0], [-0.03, 0.98, -10.0], [1e-5, 2e-5, 1.0]])


def feature_pair_problem(na: int, nb: int, seed: int = 9, kind: str = "hamming", match_frac: float = 0.6,
                         sigma: float = 0.5, H: np.ndarray = H_PIX, size=(640.0, 480.0)):
    """Two 'images' of keypoints + descriptors: a fraction of a's keypoints reappear in b at
    H(a) + N(0, sigma) px with a perturbed copy of their descriptor (binary: bit flips; SIFT-like:
    additive noise); the rest of b is random. -> (pts_a, desc_a, pts_b, desc_b, planted)"""
    rng = np.random.default_rng(seed)
    if kind == "hamming":
        da, db, planted = hamming_problem(na, nb, seed=seed, random_frac=1.0 - match_frac)
    else:
        da, db, planted = l2_problem(na, nb, seed=seed, random_frac=1.0 - match_frac)
    pa = rng.uniform([0, 0], size, size=(na, 2))
    pb = rng.uniform([0, 0], size, size=(nb, 2))
    ok = planted >= 0
    pb[planted[ok]] = project(H, pa[ok]) + rng.normal(0, sigma, size=(int(ok.sum()), 2))
    return pa, da, pb, db, planted


def scaled_problem(n: int, seed: int = 10, outlier_frac: float = 0.3, sigma: float = 1e-3, true_scale: float = 2.5,
                   focal=(1.0, 1.0)):
    """CameraPose.findScaled inputs: a lookAt source camera (Camera.fs:93-104), a
    relative pose (rotation, unit translation) and world points seen by the destination camera
    transformedView (transformation (scale true_scale pose)) srcCam; observations = project1 of
    that camera (Camera.fs:72-83) + N(0, sigma), a fraction replaced by uniform [-1, 1]^2 outliers.
    -> (srcCam, pose, world[n,3], obs[n,2], is_inlier)"""
    from . import camera as CM
    rng = np.random.default_rng(seed)
    src = CM.lookAt([0.0, -10.0, 1.0], [0.0, 0.0, 0.0], [0.0, 0.0, 1.0], focal)
    R = rotation([0.2, 0.3, 1.0], np.deg2rad(12.0))
    t = np.array([0.6, 0.1, -0.2])
    t = t / np.linalg.norm(t)
    pose = CM.CameraPose(1, 1, R, t, False)
    dst = CM.transformed_view(CM.transformation(CM.scale(true_scale, pose)), src)
    world = np.empty((0, 3))
    while world.shape[0] < n:
        w = rng.uniform(-3, 3, size=(4 * n, 3))
        _, v1 = CM.project1(dst, w)
        _, v0 = CM.project1(src, w)
        world = np.concatenate([world, w[v1 & v0]])
    world = world[:n]
    obs, _ = CM.project1(dst, world)
    obs = obs + rng.normal(0, sigma, size=obs.shape)
    out = rng.random(n) < outlier_frac
    obs[out] = rng.uniform(-1, 1, size=(int(out.sum()), 2))
    return src, pose, world, obs, ~out
