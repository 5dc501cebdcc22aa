"""Certified packed-fp32 Sampson prefilter (minicv_amd/csrc/sampson_pk.h) through its host twin: every
lane it decides must equal the exact fp64 Sampson test (hyp_fundamental.h f_error, kinds 0 / 1), on the
true model, perturbed and random models, with points crafted onto the threshold (Sampson error within
1e-7 relative of thr^2). CPU only (the GPU sweeps' counts are checked against the oracle in
test_gpu_fundamental.py / test_gpu_essential.py)."""
import numpy as np
import pytest

from minicv_amd import synthetic as S


def _cert(L, pts4, F, thr2, kind):
    n = pts4.shape[0]
    dec = np.zeros(n, np.int32)
    ex = np.zeros(n, np.int32)
    F9 = np.ascontiguousarray(F, np.float64).ravel()
    bad = L.mcvHostSampsonCert(pts4.ctypes.data, n, F9.ctypes.data, thr2, kind, dec.ctypes.data, ex.ctypes.data)
    return bad, dec, ex


def _sampson(F, x1, x2):
    X1 = np.c_[x1, np.ones(len(x1))]
    X2 = np.c_[x2, np.ones(len(x2))]
    Fx1 = X1 @ F.T
    Ftx2 = X2 @ F
    c = np.sum(X2 * Fx1, 1)
    den = Fx1[:, 0] ** 2 + Fx1[:, 1] ** 2 + Ftx2[:, 0] ** 2 + Ftx2[:, 1] ** 2
    return c * c / den


def _on_threshold(F, x1, x2, thr2, rng):
    """Move x2 along the epipolar line's normal until the Sampson error is thr2 (bisection in fp64), then
    jitter the offset by tiny relative amounts on both sides."""
    X1 = np.c_[x1, np.ones(len(x1))]
    l = X1 @ F.T
    nrm = l[:, :2] / np.linalg.norm(l[:, :2], axis=1, keepdims=True)
    c0 = np.sum(np.c_[x2, np.ones(len(x2))] * l, 1)
    base = x2 - (c0 / np.linalg.norm(l[:, :2], axis=1))[:, None] * nrm      # on the epipolar line
    lo, hi = np.zeros(len(x1)), np.full(len(x1), 1.0)
    for _ in range(200):
        mid = (lo + hi) / 2
        e = _sampson(F, x1, base + mid[:, None] * nrm)
        lo = np.where(e < thr2, mid, lo)
        hi = np.where(e < thr2, hi, mid)
    t = lo * (1 + rng.choice([-1e-6, -1e-7, 0.0, 1e-7, 1e-6, 1e-3], len(x1)))
    return base + t[:, None] * nrm


@pytest.mark.parametrize("kind", [0, 1])
def test_sampson_cert_decisions_equal_exact(native, kind):
    L = native.lib()
    src, dst, inl, F = S.fundamental_problem(4000, 5)[:4]
    F = np.asarray(F, np.float64).reshape(3, 3)
    rng = np.random.default_rng(7)
    thr = 5e-3
    thr2 = np.float32(thr * thr)
    models = [F]
    for _ in range(10):
        models.append(F + rng.normal(size=(3, 3)) * 1e-3 * np.linalg.norm(F))
    for _ in range(10):
        G = rng.normal(size=(3, 3))
        models.append(G / np.linalg.norm(G))
    total = und = 0
    for G in models:
        ring = _on_threshold(G, src, dst, float(thr2), rng)
        for x2 in (dst, ring):
            pts4 = np.ascontiguousarray(np.c_[src, x2], np.float32)
            bad, dec, ex = _cert(L, pts4, G, thr2, kind)
            assert bad == 0, f"{bad} decided points differ from the exact fp64 test"
            total += len(dec)
            und += int((dec < 0).sum())
    # the true model on the bench-like data: essentially everything decided
    pts4 = np.ascontiguousarray(np.c_[src, dst], np.float32)
    _, dec, _ = _cert(L, pts4, F, thr2, kind)
    assert (dec < 0).mean() < 1e-3
    assert und < total   # the crafted rings leave undecided points, but not all


def test_sampson_cert_edge_inputs(native):
    L = native.lib()
    src, dst, inl, F = S.fundamental_problem(500, 6)[:4]
    F = np.asarray(F, np.float64).reshape(3, 3)
    pts4 = np.ascontiguousarray(np.c_[src, dst], np.float32)
    pts4[3] = np.nan
    pts4[7, 2] = np.inf
    thr2 = np.float32(2.5e-5)
    bad, dec, ex = _cert(L, pts4, F, thr2, 1)
    assert bad == 0
    assert (dec == -1).all()      # a non-finite point set leaves the bound's domain: nothing decided
    dummy = np.array([[0, 0, 1.0], [0, 0, 0], [0, 0, 1e10]])   # the sweep's padding model
    pts4 = np.ascontiguousarray(np.c_[src, dst], np.float32)
    bad, dec, ex = _cert(L, pts4, dummy, thr2, 1)
    assert bad == 0 and (dec == 0).all()


@pytest.mark.parametrize("kind", [0, 1])
def test_sampson_cert_near_epipoles(native, kind):
    """the outlier cut c^2 > den aout + bout where den is close to 0 (both points near their
    epipoles, so F x1 and F^T x2 nearly vanish) and the constant term bout dominates: offsets from the
    epipoles swept over 12 decades put c^2 on both sides of bout. Every decided lane must equal the exact
    test."""
    L = native.lib()
    rng = np.random.default_rng(11)
    thr2 = np.float32(5e-3 * 5e-3)
    decided = 0
    for trial in range(12):
        G = rng.normal(size=(3, 3))
        U, s, Vt = np.linalg.svd(G)
        s[2] = 0
        F = U @ np.diag(s) @ Vt
        F /= np.linalg.norm(F)
        e1, e2 = Vt[2], U[:, 2]               # F e1 = 0, e2^T F = 0
        if abs(e1[2]) < 1e-3 or abs(e2[2]) < 1e-3:
            continue
        e1, e2 = e1[:2] / e1[2], e2[:2] / e2[2]
        if np.abs(np.r_[e1, e2]).max() > 50:
            continue
        n = 4000
        scale = 10.0 ** rng.uniform(-10, 1, size=(n, 1))
        x1 = e1 + scale * rng.normal(size=(n, 2))
        x2 = e2 + scale * rng.normal(size=(n, 2)) * 10.0 ** rng.uniform(-2, 2, size=(n, 1))
        pts4 = np.ascontiguousarray(np.c_[x1, x2], np.float32)
        bad, dec, ex = _cert(L, pts4, F, thr2, kind)
        assert bad == 0, f"trial {trial}: {bad} decided points differ from the exact fp64 test"
        decided += int((dec >= 0).sum())
    assert decided > 0
