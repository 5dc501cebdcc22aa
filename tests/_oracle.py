"""ctypes loader of oracle/liboracle.so — the CPU restatement used as the parity checker.
Test infrastructure only (also imported by bench.py's cpu_baseline leg and smoke())."""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
ORACLE_DIR = ROOT / "oracle"
ORACLE_SO = ORACLE_DIR / "liboracle.so"

_P, _I, _I64, _U64, _D, _F = C.c_void_p, C.c_int, C.c_int64, C.c_uint64, C.c_double, C.c_float
_SIGS = {
    "orc_philox": (None, [_P, _P, _P]),
    "orc_set_fast_minimal": (None, [_I]),
    "orc_cv_subsets": (_I64, [_I, _P, _I, _I, _I64, _P]),
    "orc_fp_coeff_matrix": (None, [_P, _P]),
    "orc_fp_det_coeffs": (None, [_P, _P]),
    "orc_cv_begin": (_P, [_I, _I, _P, _I, _I, _I64]),
    "orc_cv_end": (None, [_P]),
    "orc_h_hypothesis": (_I, [_P, _I, _U64, _I64, _P, _P, _P]),
    "orc_h_count": (_I, [_P, _I, _P, _F, _P, _I]),
    "orc_h_counts": (None, [_P, _I, _U64, _I64, _I64, _F, _I, _P, _I]),
    "orc_update_num_iters": (_I, [_D, _D, _I, _I]),
    "orc_ransac_replay": (_I64, [_P, _I64, _I, _I, _D, _I, _I, _P]),
    "orc_find_homography": (_I, [_P, _P, _I, _D, _D, _I, _I, _U64, _I, _P, _P, _P, _I]),
    "orc_match_hamming": (None, [_P, _I, _P, _I, _I, _P, _P, _P, _P, _I]),
    "orc_match_l2": (None, [_P, _I, _P, _I, _I, _P, _P, _P, _P, _I]),
    "orc_max_threads": (_I, []),
    "orc_f_hypothesis": (_I, [_P, _I, _U64, _I64, _P, _P]),
    "orc_f_count": (_I, [_P, _I, _P, _F, _I, _P]),
    "orc_f_counts": (None, [_P, _I, _U64, _I64, _I64, _F, _I, _P, _I]),
    "orc_find_fundamental": (_I, [_P, _P, _I, _D, _D, _I, _I, _U64, _I, _I, _P, _P, _P, _I]),
    "orc_poly_real_roots": (_I, [_P, _I, _P]),
    "orc_e_solve5": (_I, [_P, _P, _P, _P, _P]),
    "orc_f7_solve": (_I, [_P, _P, _P, _P, _P]),
    "orc_f7_hypothesis": (_I, [_P, _I, _U64, _I64, _P, _P]),
    "orc_f7_counts": (None, [_P, _I, _U64, _I64, _I64, _F, _I, _P, _I]),
    "orc_find_fundamental7": (_I, [_P, _P, _I, _D, _D, _I, _U64, _I, _I, _P, _P, _P, _I]),
    "orc_e_solve5_ref": (_I, [_P, _P, _P, _P, _P]),
    "orc_solve_poly10": (None, [_P, _P, _P]),
    "orc_e_hypothesis": (_I, [_P, _I, _U64, _I64, _P, _P]),
    "orc_e_count": (_I, [_P, _I, _P, _F, _I, _P]),
    "orc_e_counts": (None, [_P, _I, _U64, _I64, _I64, _F, _I, _P, _I]),
    "orc_ransac_replay_slots": (_I64, [_P, _I64, _I, _I, _I, _D, _I, _I, _P]),
    "orc_find_essential": (_I, [_P, _P, _I, _D, _D, _D, _D, _D, _I, _U64, _I, _P, _P, _P, _I]),
    "orc_e_decompose": (None, [_P, _P, _P, _P]),
    "orc_recover_pose": (_I, [_P, _P, _I, _D, _D, _D, _P, _P, _P, _P, _P]),
    "orc_ap3p_poses": (_I, [_P, _P, _P, _P]),
    "orc_solve_ap3p": (_I, [_P, _P, _P, _D, _D, _D, _D, _P, _P]),
    "orc_libm": (_I, [_I, _P, _P, _I, _P]),
    "orc_ap3p_last_branch": (_I, []),
    "orc_pnp_hypothesis": (_I, [_P, _I, _P, _U64, _I64, _P, _P, _P]),
    "orc_pnp_count": (_I, [_P, _I, _P, _P, _P, _F, _I, _P]),
    "orc_pnp_counts": (None, [_P, _I, _P, _U64, _I64, _I64, _F, _I, _P, _I]),
    "orc_pnp_lm": (None, [_P, _I, _P, _P, _P, _P, _I]),
    "orc_solve_pnp_ransac": (_I, [_P, _P, _I, _P, _P, _D, _D, _I, _U64, _I, _P, _P, _P, _P, _I]),
    "orc_pnp_vvs": (None, [_P, _I, _P, _P, _P, _I, _D]),
    "orc_pnp_counts_k": (None, [_P, _I, _P, _U64, _I64, _I64, _F, _I, _I, _P, _I]),
    "orc_solve_pnp_ransac_k": (_I, [_P, _P, _I, _P, _P, _D, _D, _I, _U64, _I, _I, _P, _P, _P, _P, _I]),
    "orc_solve_pnp": (_I, [_P, _P, _I, _P, _P, _I, _P, _P]),
    "orc_sqpnp_pose": (_I, [_P, _P, _I, _P, _P, _P]),
    "orc_epnp": (None, [_P, _P, _I, _P, _P, _P]),
    "orc_epnp5_f32": (None, [_P, _P, _P, _P]),
    "orc_pnp_hypothesis_epnp": (_I, [_P, _I, _P, _U64, _I64, _P, _P, _P]),
    "orc_epnp_points": (None, [_P, _P, _I, _P, _P, _P]),
    "orc_rodrigues": (None, [_P, _P, _P]),
    "orc_rodrigues_inv": (None, [_P, _P]),
    "orc_scaled_costs": (None, [_P, _P, _P, _I, _P, _P, _P, _P, _P, _I]),
    "orc_find_scaled": (_I, [_P, _P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _I]),
    "orc_scaled_costs_sample": (None, [_P, _P, _P, _I, _P, _P, _I, _P, _P, _P, _I]),
}

_lib = None


def load() -> C.CDLL:
    global _lib
    if _lib is None:
        srcs = [ORACLE_DIR / n for n in ("oracle.c", "oracle_e.c", "oracle_pnp.c", "oracle_epnp.c", "oracle_f7.c",
                                          "oracle_scaled.c", "oracle_int.h", "fivepoint_terms.inc")]
        if not ORACLE_SO.exists() or ORACLE_SO.stat().st_mtime < max(p.stat().st_mtime for p in srcs):
            subprocess.run(["make", "-C", str(ORACLE_DIR)], check=True, capture_output=True)
        L = C.CDLL(str(ORACLE_SO))
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _lib = L
    return _lib


class fast_minimal:
    """Context: the MCV_FLAG_FAST_MINIMAL replacement minimal solvers (H / 8-point F elimination, E Illinois,
    AP3P real-root finder)."""

    def __init__(self, on: bool = True):
        self.on = on

    def __enter__(self):
        load().orc_set_fast_minimal(int(self.on))
        return self

    def __exit__(self, *exc):
        load().orc_set_fast_minimal(0)


def cv_subsets(check: int, pts4, n: int, m: int, rows: int):
    """OpenCV's getSubset stream (check 0 none, 1 homography, 2 fundamental) -> (accepted rows, int32[rows, m])."""
    out = np.zeros((max(rows, 1), m), dtype=np.int32)
    p = 0 if pts4 is None else ptr(np.ascontiguousarray(pts4, dtype=np.float32))
    k = load().orc_cv_subsets(check, p, n, m, rows, ptr(out))
    return int(k), out[:rows]


class cv_stream:
    """Context: the oracle's hypothesis functions take OpenCV's sample stream (check 0 / 1 / 2 as in
    cv_subsets) instead of Philox, for `rows` hypotheses."""

    def __init__(self, check: int, pts4, n: int, m: int, rows: int):
        self.args = (check, pts4, n, m, rows)
        self.h = None

    def __enter__(self):
        check, pts4, n, m, rows = self.args
        self.keep = None if pts4 is None else np.ascontiguousarray(pts4, dtype=np.float32)
        self.h = load().orc_cv_begin(32, check, 0 if self.keep is None else ptr(self.keep), n, m, rows)
        return self

    def __exit__(self, *exc):
        load().orc_cv_end(self.h)


def ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def pack4(src: np.ndarray, dst: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(np.concatenate([src, dst], axis=1).astype(np.float32))


def philox(ctr, key):
    c = np.asarray(ctr, dtype=np.uint32)
    k = np.asarray(key, dtype=np.uint32)
    o = np.zeros(4, dtype=np.uint32)
    load().orc_philox(ptr(c), ptr(k), ptr(o))
    return [int(v) for v in o]


def h_hypothesis(pts4: np.ndarray, seed: int, hyp: int):
    H = np.zeros(9)
    hf = np.zeros(8, dtype=np.float32)
    idx = np.full(4, -1, dtype=np.int32)
    st = load().orc_h_hypothesis(ptr(pts4), pts4.shape[0], seed, hyp, ptr(H), ptr(hf), ptr(idx))
    return st, H, hf, idx


def h_count(pts4: np.ndarray, hf: np.ndarray, thr2: float, want_mask: bool = False, fused: bool = False):
    hf = np.ascontiguousarray(hf, dtype=np.float32)
    m = np.zeros(pts4.shape[0], dtype=np.uint8) if want_mask else None
    n = load().orc_h_count(ptr(pts4), pts4.shape[0], ptr(hf), thr2, ptr(m) if want_mask else None, int(fused))
    return (n, m) if want_mask else n


def h_counts(pts4: np.ndarray, seed: int, begin: int, count: int, thr2: float, nthreads: int = 0,
             fused: bool = False) -> np.ndarray:
    out = np.zeros(count, dtype=np.int32)
    load().orc_h_counts(ptr(pts4), pts4.shape[0], seed, begin, count, thr2, int(fused), ptr(out), nthreads)
    return out


def find_homography(src, dst, thr=3.0, conf=0.995, max_iters=2000, method=8, seed=0, flags=0, nthreads=0):
    src = np.ascontiguousarray(src, dtype=np.float64)
    dst = np.ascontiguousarray(dst, dtype=np.float64)
    n = src.shape[0]
    H = np.zeros(9)
    mask = np.zeros(max(n, 1), dtype=np.uint8)
    best = np.zeros(1, dtype=np.int64)
    cnt = load().orc_find_homography(ptr(src), ptr(dst), n, thr, conf, max_iters, method, seed, flags, ptr(H),
                                     ptr(mask), ptr(best), nthreads)
    return cnt, H.reshape(3, 3), mask[:n], int(best[0])


def replay(counts: np.ndarray, n: int, m: int, conf: float, max_iters: int, fixed: bool):
    counts = np.ascontiguousarray(counts, dtype=np.int32)
    bc = np.zeros(1, dtype=np.int32)
    best = load().orc_ransac_replay(ptr(counts), counts.shape[0], n, m, conf, max_iters, int(fixed), ptr(bc))
    return int(best), int(bc[0])


def match_hamming(q, t, nthreads=0):
    q = np.ascontiguousarray(q, dtype=np.uint8)
    t = np.ascontiguousarray(t, dtype=np.uint8)
    nq = q.shape[0]
    out = [np.zeros(nq, dtype=np.int32) for _ in range(4)]
    load().orc_match_hamming(ptr(q), nq, ptr(t), t.shape[0], q.shape[1], *[ptr(o) for o in out], nthreads)
    return tuple(out)


def match_l2(q, t, nthreads=0):
    q = np.ascontiguousarray(q, dtype=np.float32)
    t = np.ascontiguousarray(t, dtype=np.float32)
    nq = q.shape[0]
    i1, i2 = np.zeros(nq, np.int32), np.zeros(nq, np.int32)
    d1, d2 = np.zeros(nq), np.zeros(nq)
    load().orc_match_l2(ptr(q), nq, ptr(t), t.shape[0], q.shape[1], ptr(i1), ptr(d1), ptr(i2), ptr(d2), nthreads)
    return i1, d1, i2, d2


def f_hypothesis(pts4: np.ndarray, seed: int, hyp: int):
    F = np.zeros(9)
    idx = np.full(8, -1, dtype=np.int32)
    st = load().orc_f_hypothesis(ptr(pts4), pts4.shape[0], seed, hyp, ptr(F), ptr(idx))
    return st, F, idx


def f_kind(error_kind: int = 0, unfused: bool = False) -> int:
    return (2 if error_kind == 1 else 0) + (1 if unfused else 0)


def f_count(pts4, F, thr2, kind=0, want_mask=False):
    F = np.ascontiguousarray(F, dtype=np.float64).ravel()
    m = np.zeros(pts4.shape[0], dtype=np.uint8) if want_mask else None
    n = load().orc_f_count(ptr(pts4), pts4.shape[0], ptr(F), thr2, kind, ptr(m) if want_mask else None)
    return (n, m) if want_mask else n


def f_counts(pts4, seed, begin, count, thr2, kind=1, nthreads=0):
    out = np.zeros(count, dtype=np.int32)
    load().orc_f_counts(ptr(pts4), pts4.shape[0], seed, begin, count, thr2, kind, ptr(out), nthreads)
    return out


def find_fundamental(a, b, thr=3.0, conf=0.99, max_iters=1000, method=8, seed=0, flags=0, error_kind=0, nthreads=0):
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    n = a.shape[0]
    F = np.zeros(9)
    mask = np.zeros(max(n, 1), dtype=np.uint8)
    best = np.zeros(1, dtype=np.int64)
    cnt = load().orc_find_fundamental(ptr(a), ptr(b), n, thr, conf, max_iters, method, seed, flags, error_kind,
                                      ptr(F), ptr(mask), ptr(best), nthreads)
    return cnt, F.reshape(3, 3), mask[:n], int(best[0])


# ---- essential matrix (oracle_e.c) ---------------------------------------------------------
E_SLOTS = 10


F7_SLOTS = 3


def f7_hypothesis(pts4, seed, hyp):
    """7-point hypothesis -> (n or status, F[3,3,3], idx[7])."""
    F, idx = np.zeros(27), np.full(7, -1, dtype=np.int32)
    n = load().orc_f7_hypothesis(ptr(pts4), pts4.shape[0], seed, hyp, ptr(F), ptr(idx))
    return n, F.reshape(3, 3, 3), idx


def f7_counts(pts4, seed, begin, count, thr2, kind=3, nthreads=0):
    out = np.zeros(count * F7_SLOTS, dtype=np.int32)
    load().orc_f7_counts(ptr(pts4), pts4.shape[0], seed, begin, count, thr2, kind, ptr(out), nthreads)
    return out


def find_fundamental7(a, b, thr=3.0, conf=0.99, max_iters=1000, seed=0, flags=0, error_kind=1, nthreads=0):
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    n = a.shape[0]
    F, mask, best = np.zeros(9), np.zeros(max(n, 1), dtype=np.uint8), np.zeros(1, dtype=np.int64)
    cnt = load().orc_find_fundamental7(ptr(a), ptr(b), n, thr, conf, max_iters, seed, flags, error_kind, ptr(F),
                                       ptr(mask), ptr(best), nthreads)
    return cnt, F.reshape(3, 3), mask[:n], int(best[0])


def pack_e(a, b, focal=1.0, pp=(0.0, 0.0)) -> np.ndarray:
    """double4 normalised correspondences, (x - pp) / focal in fp64 (same as mcv_e_pack)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    ppa = np.asarray(pp, dtype=np.float64)
    return np.ascontiguousarray(np.concatenate([(a - ppa) / focal, (b - ppa) / focal], axis=1))


def poly_real_roots(c):
    c = np.ascontiguousarray(c, dtype=np.float64)
    r = np.zeros(10)
    n = load().orc_poly_real_roots(ptr(c), len(c) - 1, ptr(r))
    return r[:n]


def e_solve5(x1, y1, x2, y2):
    arrs = [np.ascontiguousarray(v, dtype=np.float64) for v in (x1, y1, x2, y2)]
    E = np.zeros(90)
    n = load().orc_e_solve5(*[ptr(v) for v in arrs], ptr(E))
    return E.reshape(10, 3, 3)[:max(n, 0)]


def e_solve5_ref(x1, y1, x2, y2):
    """cvFivePoint's own path (JacobiSVD null space, LU, solvePoly, solveZ)."""
    arrs = [np.ascontiguousarray(v, dtype=np.float64) for v in (x1, y1, x2, y2)]
    E = np.zeros(90)
    n = load().orc_e_solve5_ref(*[ptr(v) for v in arrs], ptr(E))
    return E.reshape(10, 3, 3)[:max(n, 0)]


def solve_poly10(c):
    """cv::solvePoly(c ascending, 300 iterations) -> complex roots in its order."""
    c = np.ascontiguousarray(c, dtype=np.float64)
    re, im = np.zeros(10), np.zeros(10)
    load().orc_solve_poly10(ptr(c), ptr(re), ptr(im))
    return re + 1j * im


def e_hypothesis(pts4d, seed, hyp):
    E = np.zeros(90)
    idx = np.full(5, -1, dtype=np.int32)
    n = load().orc_e_hypothesis(ptr(pts4d), pts4d.shape[0], seed, hyp, ptr(E), ptr(idx))
    return n, E.reshape(10, 9), idx


def e_count(pts4d, E, thr2, kind=0, want_mask=False):
    E = np.ascontiguousarray(E, dtype=np.float64).ravel()
    m = np.zeros(pts4d.shape[0], dtype=np.uint8) if want_mask else None
    n = load().orc_e_count(ptr(pts4d), pts4d.shape[0], ptr(E), thr2, kind, ptr(m) if want_mask else None)
    return (n, m) if want_mask else n


def e_counts(pts4d, seed, begin, count, thr2, kind=1, nthreads=0):
    out = np.zeros(count * E_SLOTS, dtype=np.int32)
    load().orc_e_counts(ptr(pts4d), pts4d.shape[0], seed, begin, count, thr2, kind, ptr(out), nthreads)
    return out


def replay_slots(counts, nhyp, n, m, conf, max_iters, fixed, slots=E_SLOTS):
    counts = np.ascontiguousarray(counts, dtype=np.int32)
    bc = np.zeros(1, dtype=np.int32)
    best = load().orc_ransac_replay_slots(ptr(counts), nhyp, slots, n, m, conf, max_iters, int(fixed), ptr(bc))
    return int(best), int(bc[0])


def find_essential(a, b, focal=1.0, pp=(0.0, 0.0), thr=1.0, conf=0.999, max_iters=1000, seed=0, flags=0, nthreads=0):
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    n = a.shape[0]
    E = np.zeros(9)
    mask = np.zeros(max(n, 1), dtype=np.uint8)
    best = np.zeros(1, dtype=np.int64)
    cnt = load().orc_find_essential(ptr(a), ptr(b), n, focal, pp[0], pp[1], thr, conf, max_iters, seed, flags,
                                    ptr(E), ptr(mask), ptr(best), nthreads)
    return cnt, E.reshape(3, 3), mask[:n], int(best[0])


def e_decompose(E):
    E = np.ascontiguousarray(E, dtype=np.float64).ravel()
    R1, R2, t = np.zeros(9), np.zeros(9), np.zeros(3)
    load().orc_e_decompose(ptr(E), ptr(R1), ptr(R2), ptr(t))
    return R1.reshape(3, 3), R2.reshape(3, 3), t


def recover_pose(a, b, E, mask=None, focal=1.0, pp=(0.0, 0.0)):
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    E = np.ascontiguousarray(E, dtype=np.float64).ravel()
    m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
    R, t, g = np.zeros(9), np.zeros(3), np.zeros(4, dtype=np.int32)
    res = load().orc_recover_pose(ptr(a), ptr(b), a.shape[0], focal, pp[0], pp[1], ptr(E),
                                  None if m is None else ptr(m), ptr(R), ptr(t), ptr(g))
    return res, R.reshape(3, 3), t, g


# ---- PnP (oracle_pnp.c) ---------------------------------------------------------------------
def cam8(K, dist=None):
    K = np.asarray(K, dtype=np.float64).reshape(3, 3)
    d = np.zeros(4) if dist is None else np.asarray(dist, dtype=np.float64)
    return np.ascontiguousarray([K[0, 0], K[1, 1], K[0, 2], K[1, 2], d[0], d[1], d[2], d[3]], dtype=np.float64)


def pack_pnp(img, world) -> np.ndarray:
    """PnpPoint layout: float32 [N][8] {X, Y, Z, u, v, 0, 0, 0}."""
    img = np.asarray(img, dtype=np.float64)
    world = np.asarray(world, dtype=np.float64)
    p = np.zeros((img.shape[0], 8), dtype=np.float32)
    p[:, 0:3] = world.astype(np.float32)
    p[:, 3:5] = img.astype(np.float32)
    return np.ascontiguousarray(p)


def pnp_hypothesis(pts8, c8, seed, hyp):
    R, t, idx = np.zeros(9), np.zeros(3), np.full(4, -1, dtype=np.int32)
    st = load().orc_pnp_hypothesis(ptr(pts8), pts8.shape[0], ptr(c8), seed, hyp, ptr(R), ptr(t), ptr(idx))
    return st, R.reshape(3, 3), t, idx


def pnp_counts(pts8, c8, seed, begin, count, thr2, fused=False, nthreads=0, kind=5):
    """Per-hypothesis counts with the minimal solver of solverKind `kind` (AP3P for 2 / 5, else EPnP)."""
    out = np.zeros(count, dtype=np.int32)
    load().orc_pnp_counts_k(ptr(pts8), pts8.shape[0], ptr(c8), seed, begin, count, thr2, int(fused), int(kind),
                            ptr(out), nthreads)
    return out


def pnp_lm(pts8, c8, rvec, tvec, mask=None, max_iters=20):
    """cvRefinePnPLM's definition (pnp_host.cpp pnp_lm) -> (rvec, tvec)."""
    r = np.ascontiguousarray(rvec, dtype=np.float64).copy()
    t = np.ascontiguousarray(tvec, dtype=np.float64).copy()
    m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
    load().orc_pnp_lm(ptr(pts8), pts8.shape[0], None if m is None else ptr(m), ptr(c8), ptr(r), ptr(t), max_iters)
    return r, t


def pnp_vvs(pts8, c8, rvec, tvec, max_iters=20, lam=1.0):
    """cvRefinePnPVVS's definition (pnp_host.cpp pnp_vvs) -> (rvec, tvec)."""
    r = np.ascontiguousarray(rvec, dtype=np.float64).copy()
    t = np.ascontiguousarray(tvec, dtype=np.float64).copy()
    load().orc_pnp_vvs(ptr(pts8), pts8.shape[0], ptr(c8), ptr(r), ptr(t), max_iters, lam)
    return r, t


def pnp_hypothesis_epnp(pts8, c8, seed, hyp):
    R, t, idx = np.zeros(9), np.zeros(3), np.full(5, -1, dtype=np.int32)
    st = load().orc_pnp_hypothesis_epnp(ptr(pts8), pts8.shape[0], ptr(c8), seed, hyp, ptr(R), ptr(t), ptr(idx))
    return st, R.reshape(3, 3), t, idx


def epnp(pw, us, cam4):
    """compute_pose on n points: pw (n, 3) world, us (n, 2) pixels, cam4 = (fu, fv, uc, vc)."""
    pw = np.ascontiguousarray(pw, dtype=np.float64)
    us = np.ascontiguousarray(us, dtype=np.float64)
    c = np.ascontiguousarray(cam4, dtype=np.float64)
    R, t = np.zeros(9), np.zeros(3)
    load().orc_epnp(ptr(pw), ptr(us), pw.shape[0], ptr(c), ptr(R), ptr(t))
    return R.reshape(3, 3), t


def epnp_points(img, world, c8):
    """solvePnP(EPNP) on double points: undistortPoints (double) then compute_pose."""
    img = np.ascontiguousarray(img, dtype=np.float64)
    world = np.ascontiguousarray(world, dtype=np.float64)
    R, t = np.zeros(9), np.zeros(3)
    load().orc_epnp_points(ptr(img), ptr(world), img.shape[0], ptr(np.ascontiguousarray(c8, dtype=np.float64)),
                           ptr(R), ptr(t))
    return R.reshape(3, 3), t


def solve_pnp(img, world, K, dist=None, kind=1):
    """cvSolvePnP for kinds 0 / 1 / 3 / 4 / 6 -> (ok, rvec, tvec)."""
    img = np.ascontiguousarray(img, dtype=np.float64)
    world = np.ascontiguousarray(world, dtype=np.float64)
    K9 = np.ascontiguousarray(np.asarray(K, dtype=np.float64).ravel())
    d = np.ascontiguousarray(np.zeros(4) if dist is None else np.asarray(dist, dtype=np.float64))
    r, t = np.zeros(3), np.zeros(3)
    ok = load().orc_solve_pnp(ptr(img), ptr(world), img.shape[0], ptr(K9), ptr(d), int(kind), ptr(r), ptr(t))
    return bool(ok), r, t


def sqpnp_pose(img, world, cam8):
    """oracle_sqpnp.c's solve -> (code, R (3 x 3), t): code > 0 = solution count."""
    img = np.ascontiguousarray(img, dtype=np.float64)
    world = np.ascontiguousarray(world, dtype=np.float64)
    c8 = np.ascontiguousarray(cam8, dtype=np.float64)
    R, t = np.zeros(9), np.zeros(3)
    code = load().orc_sqpnp_pose(ptr(img), ptr(world), img.shape[0], ptr(c8), ptr(R), ptr(t))
    return code, R.reshape(3, 3), t


def pnp_count(pts8, c8, R, t, thr2, fused=False):
    R = np.ascontiguousarray(R, dtype=np.float64).ravel()
    t = np.ascontiguousarray(t, dtype=np.float64)
    m = np.zeros(pts8.shape[0], dtype=np.uint8)
    n = load().orc_pnp_count(ptr(pts8), pts8.shape[0], ptr(c8), ptr(R), ptr(t), thr2, int(fused), ptr(m))
    return n, m


def solve_pnp_ransac(img, world, K, dist=None, thr=8.0, conf=0.99, max_iters=100, seed=0, flags=0, nthreads=0, kind=5):
    img = np.ascontiguousarray(img, dtype=np.float64)
    world = np.ascontiguousarray(world, dtype=np.float64)
    K9 = np.ascontiguousarray(np.asarray(K, dtype=np.float64).ravel())
    d = np.ascontiguousarray(np.zeros(4) if dist is None else np.asarray(dist, dtype=np.float64))
    n = img.shape[0]
    r, t = np.zeros(3), np.zeros(3)
    mask = np.zeros(max(n, 1), dtype=np.uint8)
    best = np.zeros(1, dtype=np.int64)
    cnt = load().orc_solve_pnp_ransac_k(ptr(img), ptr(world), n, ptr(K9), ptr(d), float(thr), conf, max_iters, seed,
                                        flags, int(kind), ptr(r), ptr(t), ptr(mask), ptr(best), nthreads)
    return cnt, r, t, mask[:n], int(best[0])


def solve_ap3p(mu, mv, W, inv_fx, inv_fy, cx_fx, cy_fy):
    mu = np.ascontiguousarray(mu, dtype=np.float64)
    mv = np.ascontiguousarray(mv, dtype=np.float64)
    W = np.ascontiguousarray(np.asarray(W, dtype=np.float64).ravel())
    Rs, ts = np.zeros(36), np.zeros(12)
    n = load().orc_solve_ap3p(ptr(mu), ptr(mv), ptr(W), inv_fx, inv_fy, cx_fx, cy_fy, ptr(Rs), ptr(ts))
    return [(Rs[9 * i:9 * i + 9].reshape(3, 3), ts[3 * i:3 * i + 3]) for i in range(n)]


def rodrigues(r):
    r = np.ascontiguousarray(r, dtype=np.float64)
    R, dR = np.zeros(9), np.zeros(27)
    load().orc_rodrigues(ptr(r), ptr(R), ptr(dR))
    return R.reshape(3, 3), dR.reshape(3, 3, 3)


def rodrigues_inv(R):
    R = np.ascontiguousarray(np.asarray(R, dtype=np.float64).ravel())
    r = np.zeros(3)
    load().orc_rodrigues_inv(ptr(R), ptr(r))
    return r


def _scaled_args(cam14, world, obs, R, t):
    cam = np.ascontiguousarray(cam14, np.float64).reshape(14)
    W = np.ascontiguousarray(world, np.float64).reshape(-1, 3)
    O = np.ascontiguousarray(obs, np.float64).reshape(-1, 2)
    R9 = np.ascontiguousarray(R, np.float64).reshape(9)
    T3 = np.ascontiguousarray(t, np.float64).reshape(3)
    return cam, W, O, R9, T3


def scaled_costs(cam14, world, obs, R, t, nthreads=0):
    """CameraPose.findScaled candidates: (scales[2N], costs[2N], used[N])."""
    cam, W, O, R9, T3 = _scaled_args(cam14, world, obs, R, t)
    n = W.shape[0]
    sc = np.empty(2 * n)
    co = np.empty(2 * n)
    used = np.zeros(n, np.uint8)
    load().orc_scaled_costs(ptr(cam), ptr(W), ptr(O), n, ptr(R9), ptr(T3), ptr(sc), ptr(co), ptr(used), nthreads)
    return sc, co, used


def find_scaled(cam14, world, obs, R, t, nthreads=0):
    """CameraPose.findScaled: (cost, scale, evaluated candidates)."""
    cam, W, O, R9, T3 = _scaled_args(cam14, world, obs, R, t)
    n = W.shape[0]
    sc = np.empty(max(2 * n, 1))
    co = np.empty(max(2 * n, 1))
    used = np.zeros(max(n, 1), np.uint8)
    cost, scale = C.c_double(0), C.c_double(0)
    k = load().orc_find_scaled(ptr(cam), ptr(W), ptr(O), n, ptr(R9), ptr(T3), ptr(sc), ptr(co), ptr(used),
                               C.addressof(cost), C.addressof(scale), nthreads)
    return cost.value, scale.value, k


def scaled_costs_sample(cam14, world, obs, R, t, n_cand, nthreads=0):
    """Costs of the first n_cand candidates (CPU baseline sample)."""
    cam, W, O, R9, T3 = _scaled_args(cam14, world, obs, R, t)
    n = W.shape[0]
    sc, co, used = np.empty(2 * n), np.empty(2 * n), np.zeros(n, np.uint8)
    load().orc_scaled_costs_sample(ptr(cam), ptr(W), ptr(O), n, ptr(R9), ptr(T3), n_cand, ptr(sc), ptr(co),
                                   ptr(used), nthreads)
    return co[:n_cand]


def libm(fn, a, b=None):
    """glibc's cbrt (fn 0), hypot (1), creal(clog(a + i b)) (2), exp (4), log (5), log1p (6), cos (7) or
    atan2(a, b) (8) over arrays, from the oracle library."""
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(a if b is None else b, dtype=np.float64)
    out = np.zeros_like(a)
    assert load().orc_libm(fn, ptr(a), ptr(b), a.shape[0], ptr(out)) == a.shape[0]
    return out


def ap3p_last_branch():
    """The branch the oracle's last Ferrari quartic took: 0 real w (cbrt), 1 complex w (pow), -1 none."""
    return load().orc_ap3p_last_branch()
