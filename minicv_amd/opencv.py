"""Host-side mirror of the reference's managed wrappers (module `OpenCV`,
/root/reference/src/MiniCV/OpenCV.fs:855-1052): allocate caller-owned outputs, call the native
export, map the byte mask to bool, return tuples. New wrappers for the hot-path exports follow
the pattern of `OpenCV.recoverPose` (OpenCV.fs:855-861).

Everything here calls libMiniCVNative.so; errors surface as NativeError with the native message.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import native as N


@dataclass
class RansacParams:
    """RANSAC configuration (C struct RansacConfig). Defaults follow cv::findHomography
    (thr 3, maxIters 2000, confidence 0.995)."""
    threshold: float = 3.0
    confidence: float = 0.995
    max_iters: int = 2000
    method: int = N.METHOD_RANSAC
    seed: int = 0
    device_count: int = 1
    fixed_iters: bool = False
    refine: bool = True
    error_kind: int = N.FERR_SAMPSON
    fused_error: bool = False   # opt-in FMA-contracted error (default: OpenCV op-by-op order)
    seven_point: bool = False   # fundamental: OpenCV FM_RANSAC's 7-point minimal sets (<= 3 models each)
    fast_minimal: bool = False  # opt-in: H / 8-point F minimal solve by elimination (default: cv::eigen)
    cv_sampler: bool = False    # OpenCV's own sample stream (cv::RNG((uint64)-1) + getSubset); seed unused

    def to_c(self) -> N.RansacConfig:
        flags = (N.FLAG_FIXED_ITERS if self.fixed_iters else 0) | (0 if self.refine else N.FLAG_NO_REFINE) | \
            (N.FLAG_FUSED_ERROR if self.fused_error else 0) | (N.FLAG_SEVEN_POINT if self.seven_point else 0) | \
            (N.FLAG_FAST_MINIMAL if self.fast_minimal else 0) | (N.FLAG_CV_SAMPLER if self.cv_sampler else 0)
        return N.RansacConfig(self.threshold, self.confidence, int(self.max_iters), int(self.method),
                              int(self.seed) & 0xFFFFFFFFFFFFFFFF, int(self.device_count), flags,
                              int(self.error_kind), 0)


def _v2d(a) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    if a.ndim != 2 or a.shape[1] != 2:
        raise ValueError("points must be an (N, 2) array")
    return a


def findHomography(src, dst, params: RansacParams | None = None):
    """-> (inlierCount, H (3x3 float64), mask (bool[N])). Raises NativeError on failure."""
    params = params or RansacParams()
    a, b = _v2d(src), _v2d(dst)
    n = a.shape[0]
    if b.shape[0] != n:
        raise ValueError("src/dst length mismatch")
    H = N.M33d()
    ms = np.zeros(max(n, 1), dtype=np.uint8)
    cfg = params.to_c()
    cnt = N.lib().cvFindHomography(a.ctypes.data, b.ctypes.data, n, N.C.addressof(cfg), N.C.addressof(H),
                                   ms.ctypes.data)
    N.check(cnt > 0, "cvFindHomography")
    return cnt, np.array(H.M[:], dtype=np.float64).reshape(3, 3), ms[:n] != 0


def findFundamentalMat(a, b, params: RansacParams | None = None):
    """8-point RANSAC (default), or OpenCV FM_RANSAC with params.seven_point (+ error_kind EPIPOLAR).
    -> (inlierCount, F (3x3 float64), mask (bool[N]))."""
    params = params or RansacParams(threshold=3.0, confidence=0.99)
    pa, pb = _v2d(a), _v2d(b)
    n = pa.shape[0]
    F = N.M33d()
    ms = np.zeros(max(n, 1), dtype=np.uint8)
    cfg = params.to_c()
    cnt = N.lib().cvFindFundamentalMat(pa.ctypes.data, pb.ctypes.data, n, N.C.addressof(cfg), N.C.addressof(F),
                                       ms.ctypes.data)
    N.check(cnt > 0, "cvFindFundamentalMat")
    return cnt, np.array(F.M[:], dtype=np.float64).reshape(3, 3), ms[:n] != 0


def matchHamming(q, t, deviceCount: int = 1):
    """BFMatcher(NORM_HAMMING).knnMatch(k=2). q, t: uint8 [n][bytes]. -> (idx, dist, idx2, dist2).
    deviceCount > 1: cvMatchHammingMulti (query blocks over the visible GPUs, same answer)."""
    q = np.ascontiguousarray(q, dtype=np.uint8)
    t = np.ascontiguousarray(t, dtype=np.uint8)
    if q.ndim != 2 or t.ndim != 2 or q.shape[1] != t.shape[1]:
        raise ValueError("descriptor arrays must be [n][bytes] with equal widths")
    nq, nt, nb = q.shape[0], t.shape[0], q.shape[1]
    out = [np.empty(max(nq, 1), dtype=np.int32) for _ in range(4)]
    if deviceCount == 1:
        r = N.lib().cvMatchHamming(q.ctypes.data, nq, t.ctypes.data, nt, nb, *[o.ctypes.data for o in out])
    else:
        r = N.lib().cvMatchHammingMulti(q.ctypes.data, nq, t.ctypes.data, nt, nb, int(deviceCount),
                                        *[o.ctypes.data for o in out])
    N.check(r == nq, "cvMatchHamming")
    return tuple(o[:nq] for o in out)


def matchL2(q, t, deviceCount: int = 1):
    """BFMatcher(NORM_L2).knnMatch(k=2). q, t: float32 [n][dim]. -> (idx, dist, idx2, dist2).
    deviceCount > 1: cvMatchL2Multi (query blocks over the visible GPUs, same answer)."""
    q = np.ascontiguousarray(q, dtype=np.float32)
    t = np.ascontiguousarray(t, dtype=np.float32)
    if q.ndim != 2 or t.ndim != 2 or q.shape[1] != t.shape[1]:
        raise ValueError("descriptor arrays must be [n][dim] with equal widths")
    nq, nt, dim = q.shape[0], t.shape[0], q.shape[1]
    idx, idx2 = np.empty(max(nq, 1), np.int32), np.empty(max(nq, 1), np.int32)
    d, d2 = np.empty(max(nq, 1), np.float32), np.empty(max(nq, 1), np.float32)
    if deviceCount == 1:
        r = N.lib().cvMatchL2(q.ctypes.data, nq, t.ctypes.data, nt, dim, idx.ctypes.data, d.ctypes.data,
                              idx2.ctypes.data, d2.ctypes.data)
    else:
        r = N.lib().cvMatchL2Multi(q.ctypes.data, nq, t.ctypes.data, nt, dim, int(deviceCount), idx.ctypes.data,
                                   d.ctypes.data, idx2.ctypes.data, d2.ctypes.data)
    N.check(r == nq, "cvMatchL2")
    return idx[:nq], d[:nq], idx2[:nq], d2[:nq]


def recoverPoseConfig(focal: float = 1.0, pp=(0.0, 0.0), probability: float = 0.999,
                      threshold: float = 0.005) -> N.RecoverPoseConfig:
    """RecoverPoseConfig (OpenCV.fs:16-36); defaults = RecoverPoseConfig.Default (:33-34)."""
    return N.RecoverPoseConfig(float(focal), N.V2d(float(pp[0]), float(pp[1])), float(probability), float(threshold))


def findEssentialMat(a, b, focal: float = 1.0, pp=(0.0, 0.0), params: RansacParams | None = None):
    """cv::findEssentialMat(a, b, focal, pp, RANSAC, ...) on the GPU.
    -> (inlierCount, E (3x3 float64, unit Frobenius norm), mask (bool[N]))."""
    params = params or RansacParams(threshold=1.0, confidence=0.999, max_iters=1000)
    pa, pb = _v2d(a), _v2d(b)
    n = pa.shape[0]
    if pb.shape[0] != n:
        raise ValueError("a/b length mismatch")
    E = N.M33d()
    ms = np.zeros(max(n, 1), dtype=np.uint8)
    cfg = params.to_c()
    cnt = N.lib().cvFindEssentialMat(pa.ctypes.data, pb.ctypes.data, n, float(focal), N.V2d(*map(float, pp)),
                                     N.C.addressof(cfg), N.C.addressof(E), ms.ctypes.data)
    N.check(cnt > 0, "cvFindEssentialMat")
    return cnt, np.array(E.M[:], dtype=np.float64).reshape(3, 3), ms[:n] != 0


def recoverPose(cfg: N.RecoverPoseConfig, a, b):
    """OpenCV.recoverPose (OpenCV.fs:855-861): -> (res, R, t, mask bytes). res is the number of
    RANSAC inliers passing the cheirality test; the mask is the RANSAC mask (MiniCVNative.cpp:206-210).
    Raises NativeError when the export reports an error (the reference would throw inside OpenCV)."""
    pa, pb = _v2d(a), _v2d(b)
    m, t = N.M33d(), N.V3d(100, 123, 432)
    ms = np.zeros(max(pa.shape[0], 1), dtype=np.uint8)
    res = N.lib().cvRecoverPose(N.C.addressof(cfg), pa.shape[0], pa.ctypes.data, pb.ctypes.data,
                                N.C.addressof(m), N.C.addressof(t), ms.ctypes.data)
    if res <= 0 and N.last_error():
        raise N.NativeError(f"cvRecoverPose: {N.last_error()}")
    return res, np.array(m.M[:]).reshape(3, 3), np.array([t.X, t.Y, t.Z]), ms[:pa.shape[0]]


def recoverPoses(cfg: N.RecoverPoseConfig, a, b):
    """OpenCV.recoverPoses (OpenCV.fs:863-870): -> (R1, R2, t, mask bytes); the bool result is
    ignored like the F# wrapper does (outputs keep their initial values on failure)."""
    pa, pb = _v2d(a), _v2d(b)
    m1, m2 = N.M33d(), N.M33d()
    m1.M[:] = [1.0, 0, 0, 0, 1.0, 0, 0, 0, 1.0]
    m2.M[:] = [1.0, 0, 0, 0, 1.0, 0, 0, 0, 1.0]
    t = N.V3d(100, 123, 432)
    ms = np.zeros(max(pa.shape[0], 1), dtype=np.uint8)
    N.lib().cvRecoverPoses(N.C.addressof(cfg), pa.shape[0], pa.ctypes.data, pb.ctypes.data, N.C.addressof(m1),
                           N.C.addressof(m2), N.C.addressof(t), ms.ctypes.data)
    return (np.array(m1.M[:]).reshape(3, 3), np.array(m2.M[:]).reshape(3, 3), np.array([t.X, t.Y, t.Z]),
            ms[:pa.shape[0]])


def recoverPoses2(cfg: N.RecoverPoseConfig, a, b):
    """OpenCV.recoverPoses2 (OpenCV.fs:872-909): NDC-like input (x, y) -> (x, -y), focal and
    threshold rescaled, result mapped back with C = diag(1, -1, -1).
    -> (list of (R, t) candidate poses, mask bool[N])."""
    scale = 2.0
    pa = np.stack([(0.5 * _v2d(a)[:, 0]) * scale, (-0.5 * _v2d(a)[:, 1]) * scale], axis=1)
    pb = np.stack([(0.5 * _v2d(b)[:, 0]) * scale, (-0.5 * _v2d(b)[:, 1]) * scale], axis=1)
    c = N.RecoverPoseConfig(scale * cfg.FocalLength / 2.0, N.V2d(0.0, 0.0), cfg.Probability,
                            scale * 0.5 * cfg.InlierThreshold)
    m1, m2, t, ms = recoverPoses(c, pa, pb)
    Cm = np.diag([1.0, -1.0, -1.0])
    m1 = Cm @ m1.T @ Cm
    m2 = Cm @ m2.T @ Cm
    t = Cm @ t
    poses = [(m1, t)] if np.array_equal(m1, m2) else [(m1, t), (m2, t)]
    return poses, ms != 0


def fivepoint(a, b):
    """OpenCV.fivepoint (OpenCV.fs:912-920): -> list of up to 10 essential matrices (3x3)."""
    pa, pb = _v2d(a), _v2d(b)
    if pa.shape[0] < 5 or pb.shape[0] < 5:
        raise ValueError("fivepoint needs 5 correspondences")
    Es = (N.M33d * 10)()
    cnt = N.lib().cvFivePoint(pa.ctypes.data, pb.ctypes.data, Es)
    if cnt <= 0 and N.last_error():
        raise N.NativeError(f"cvFivePoint: {N.last_error()}")
    return [np.array(Es[i].M[:]).reshape(3, 3) for i in range(max(cnt, 0))]


# ---- PnP (OpenCV.fs:922-1052; exports MiniCVNative.cpp:48-163, ap3p.cpp:282) -----------------
SOLVER_KIND = {"Iterative": 0, "EPNP": 1, "P3P": 2, "DLS": 3, "UPNP": 4, "AP3P": 5, "SQPNP": 6}


def _m33(K) -> N.M33d:
    K = np.ascontiguousarray(np.asarray(K, dtype=np.float64).reshape(9))
    m = N.M33d()
    m.M[:] = K.tolist()
    return m


def _dist4(d):
    d = np.zeros(4) if d is None else np.ascontiguousarray(np.asarray(d, dtype=np.float64).reshape(4))
    return d


def _v3d(a) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    if a.ndim != 2 or a.shape[1] != 3:
        raise ValueError("world points must be an (N, 3) array")
    return a


def solvePnPRansac(img, world, K, dist=None, kind: str = "AP3P", iterations: int = 100, reproj_error: float = 8.0,
                   confidence: float = 0.99, params: RansacParams | None = None):
    """cvSolvePnPRansac (solvePnPInternal with `ransac`, OpenCV.fs:976-1038).
    -> (ok, rvec, tvec, inlier indices int32[count]). With `params` the seeded cvSolvePnPRansacCfg
    export is used (threshold = reprojection error in pixels)."""
    pi, pw = _v2d(img), _v3d(world)
    n = pi.shape[0]
    if pw.shape[0] != n:
        raise ValueError("img/world length mismatch")
    d = _dist4(dist)
    t, r = N.V3d(), N.V3d()
    cnt = N.C.c_int(0)
    inl = np.zeros(max(n, 1), dtype=np.int32)
    if params is None:
        ok = N.lib().cvSolvePnPRansac(pi.ctypes.data, pw.ctypes.data, n, _m33(K), d.ctypes.data, SOLVER_KIND[kind],
                                      int(iterations), float(reproj_error), float(confidence), N.C.addressof(t),
                                      N.C.addressof(r), N.C.addressof(cnt), inl.ctypes.data)
    else:
        cfg = params.to_c()
        cfg.pnpKind = SOLVER_KIND[kind]
        ok = N.lib().cvSolvePnPRansacCfg(pi.ctypes.data, pw.ctypes.data, n, _m33(K), d.ctypes.data,
                                         N.C.addressof(cfg), N.C.addressof(t), N.C.addressof(r), N.C.addressof(cnt),
                                         inl.ctypes.data)
    if not ok and N.last_error() and "no pose" not in N.last_error():
        raise N.NativeError(f"cvSolvePnPRansac: {N.last_error()}")
    return bool(ok), np.array([r.X, r.Y, r.Z]), np.array([t.X, t.Y, t.Z]), inl[:cnt.value].copy()


def solvePnP(img, world, K, dist=None, kind: str = "AP3P"):
    """cvSolvePnP -> (ok, rvec, tvec)."""
    pi, pw = _v2d(img), _v3d(world)
    d = _dist4(dist)
    t, r = N.V3d(), N.V3d()
    ok = N.lib().cvSolvePnP(pi.ctypes.data, pw.ctypes.data, pi.shape[0], _m33(K), d.ctypes.data, SOLVER_KIND[kind],
                            N.C.addressof(t), N.C.addressof(r))
    if not ok and N.last_error() and "no pose" not in N.last_error():
        raise N.NativeError(f"cvSolvePnP: {N.last_error()}")
    return bool(ok), np.array([r.X, r.Y, r.Z]), np.array([t.X, t.Y, t.Z])


def _refine(fn, img, world, K, dist, rvec, tvec):
    pi, pw = _v2d(img), _v3d(world)
    d = _dist4(dist)
    t, r = N.V3d(*map(float, tvec)), N.V3d(*map(float, rvec))
    fn(pi.ctypes.data, pw.ctypes.data, pi.shape[0], _m33(K), d.ctypes.data, N.C.addressof(t), N.C.addressof(r))
    if N.last_error():
        raise N.NativeError(N.last_error())
    return np.array([r.X, r.Y, r.Z]), np.array([t.X, t.Y, t.Z])


def refinePnPLM(img, world, K, dist, rvec, tvec):
    """cvRefinePnPLM with the given initial pose -> (rvec, tvec)."""
    return _refine(N.lib().cvRefinePnPLM, img, world, K, dist, rvec, tvec)


def refinePnPVVS(img, world, K, dist, rvec, tvec):
    """cvRefinePnPVVS -> (rvec, tvec)."""
    return _refine(N.lib().cvRefinePnPVVS, img, world, K, dist, rvec, tvec)


def solveAp3p(img, world, K):
    """OpenCV.solveAp3p (OpenCV.fs:385-431): 3 points, double arguments (F# `float` is System.Double)
    -> list of (R, t) as the reference returns them (R as stored by ap3p.cpp:245-250)."""
    img = np.asarray(img, dtype=np.float64)
    world = np.asarray(world, dtype=np.float64)
    K = np.asarray(K, dtype=np.float64).reshape(3, 3)
    Rs, ts = (N.M33d * 4)(), (N.V3d * 4)()
    inv_fx, inv_fy = 1.0 / K[0, 0], 1.0 / K[1, 1]
    args = []
    for i in range(3):
        args += [img[i, 0], img[i, 1], world[i, 0], world[i, 1], world[i, 2]]
    args += [inv_fx, inv_fy, K[0, 2] * inv_fx, K[1, 2] * inv_fy]
    cnt = N.lib().solveAp3p(Rs, ts, *[float(a) for a in args])
    if cnt <= 0 and N.last_error():
        raise N.NativeError(f"solveAp3p: {N.last_error()}")
    return [(np.array(Rs[i].M[:]).reshape(3, 3), np.array([ts[i].X, ts[i].Y, ts[i].Z])) for i in range(max(cnt, 0))]


# ---- device-resident match -> RANSAC hand-off ------------------------------
class Features:
    """A DetectorResult (MiniCVNative.h:23-29) built from keypoint coordinates and descriptors, as
    cvDetectFeatures returns it: KeyPoint2d[N] + row-major descriptors (uint8 -> Hamming,
    float32 -> L2). Keeps the backing arrays alive while the struct is in use."""

    def __init__(self, points, descriptors):
        pts = np.asarray(points, dtype=np.float64)
        d = np.ascontiguousarray(descriptors)
        if d.dtype not in (np.uint8, np.float32):
            raise ValueError("descriptors must be uint8 (Hamming) or float32 (L2)")
        n = pts.shape[0]
        self._kp = (N.KeyPoint2d * max(n, 1))()
        for i in range(n):
            self._kp[i].X, self._kp[i].Y = float(pts[i, 0]), float(pts[i, 1])
        self._d = d
        self.struct = N.DetectorResult(n, int(d.size), 0 if d.dtype == np.uint8 else 5,
                                       N.C.cast(self._kp, N.C.c_void_p), d.ctypes.data)


def _mcfg(ratio, cross_check, max_distance, model):
    return N.MatchConfig(float(ratio), int(bool(cross_check)), float(max_distance), int(model))


def matchFeatures(a: Features, b: Features, ratio: float = 0.8, cross_check: bool = False,
                  max_distance: float = 0.0):
    """cvMatchFeatures -> (pairs int32 [k][2] (index in a, index in b), dist float32 [k])."""
    n = a.struct.PointCount
    pairs = np.zeros((max(n, 1), 2), dtype=np.int32)
    dist = np.zeros(max(n, 1), dtype=np.float32)
    cfg = _mcfg(ratio, cross_check, max_distance, N.MODEL_HOMOGRAPHY)
    k = N.lib().cvMatchFeatures(N.C.addressof(a.struct), N.C.addressof(b.struct), N.C.addressof(cfg),
                                pairs.ctypes.data, dist.ctypes.data, max(n, 1))
    N.check(k >= 0, "cvMatchFeatures")
    return pairs[:k].copy(), dist[:k].copy()


def matchAndFindModel(a: Features, b: Features, model: int = N.MODEL_HOMOGRAPHY, ratio: float = 0.8,
                      cross_check: bool = False, max_distance: float = 0.0, params: RansacParams | None = None):
    """cvMatchAndFindModel -> (inliers, M 3x3, pairs [k][2], mask bool[k])."""
    n = a.struct.PointCount
    pairs = np.zeros((max(n, 1), 2), dtype=np.int32)
    mask = np.zeros(max(n, 1), dtype=np.uint8)
    M = N.M33d()
    mc = N.C.c_int(0)
    cfg = _mcfg(ratio, cross_check, max_distance, model)
    rc = (params or (RansacParams() if model == N.MODEL_HOMOGRAPHY else RansacParams(confidence=0.99))).to_c()
    cnt = N.lib().cvMatchAndFindModel(N.C.addressof(a.struct), N.C.addressof(b.struct), N.C.addressof(cfg),
                                      N.C.addressof(rc), N.C.addressof(M), pairs.ctypes.data, mask.ctypes.data,
                                      max(n, 1), N.C.addressof(mc))
    N.check(cnt > 0, "cvMatchAndFindModel")
    k = mc.value
    return cnt, np.array(M.M[:]).reshape(3, 3), pairs[:k].copy(), mask[:k] != 0
