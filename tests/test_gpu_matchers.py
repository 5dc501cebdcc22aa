"""GPU parity of the brute-force matchers against the oracle (needs an MI355X).
Hamming: integer work, bit-exact (indices, distances, second best, lowest-index tie-break).
"""
from pathlib import Path

import numpy as np
import pytest

from minicv_amd import opencv, synthetic as S

pytestmark = pytest.mark.gpu
GOLDEN = Path(__file__).resolve().parent / "golden"


def check_hamming(oracle, q, t):
    got = opencv.matchHamming(q, t)
    ref = oracle.match_hamming(q, t)
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g, r)


def test_hamming_golden(gpu):
    g = np.load(GOLDEN / "matchers.npz")
    got = opencv.matchHamming(g["hq"], g["ht"])
    for a, b in zip(got, (g["h_idx"], g["h_dist"], g["h_idx2"], g["h_dist2"])):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("nq,nt,nbytes", [(1, 1, 32), (1, 2, 32), (63, 65, 32), (1000, 777, 32), (513, 4099, 64),
                                          (300, 300, 61), (257, 1000, 16), (100, 100, 1), (2000, 3000, 32)])
def test_hamming_shapes(gpu, oracle, nq, nt, nbytes):
    q, t, _ = S.hamming_problem(nq, nt, nbytes=nbytes, seed=nq + nt)
    check_hamming(oracle, q, t)


def test_hamming_ties_lowest_index(gpu, oracle):
    rng = np.random.default_rng(1)
    base = rng.integers(0, 256, size=(50, 32), dtype=np.uint8)
    t = np.concatenate([base, base, base])           # every descriptor appears 3 times
    q = base[rng.integers(0, 50, size=400)]
    idx, dist, idx2, dist2 = opencv.matchHamming(q, t)
    assert (dist == 0).all() and (dist2 == 0).all()
    assert (idx < 50).all() and (idx2 == idx + 50).all()
    check_hamming(oracle, q, t)


def test_hamming_empty_train(gpu):
    q = np.zeros((5, 32), np.uint8)
    idx, dist, idx2, dist2 = opencv.matchHamming(q, np.zeros((0, 32), np.uint8))
    assert (idx == -1).all() and (idx2 == -1).all()


def test_hamming_cfg2_full(gpu, oracle):
    """BASELINE cfg2: 10k x 10k 256-bit ORB-like descriptors, exact against the oracle."""
    q, t, planted = S.hamming_problem(10_000, 10_000, seed=2)
    got = opencv.matchHamming(q, t)
    ref = oracle.match_hamming(q, t)
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g, r)
    ok = planted >= 0
    assert np.mean(got[0][ok] == planted[ok]) > 0.99


# ---- L2 (fp32 MFMA GEMM form) -------------------------------------------------------------
# Tolerance (north_star states 1e-6 only for H/F): the GEMM form |q|^2 + |t|^2 - 2 q.t rounds
# differently from the direct sum, so squared distances may differ by
#   tol = L2_REL * (|q|^2 + |t|^2)
# and the chosen train index may differ from the oracle's only between candidates whose exact
# squared distances are within 2 tol of each other (near-ties).
L2_REL = 2e-6


def check_l2(oracle, q, t):
    idx, d, idx2, d2 = opencv.matchL2(q, t)
    ri, rd, ri2, rd2 = oracle.match_l2(q, t)
    q64, t64 = q.astype(np.float64), t.astype(np.float64)
    qn = (q64 ** 2).sum(1)
    tn = (t64 ** 2).sum(1)
    ok = idx >= 0
    assert ok.all()
    exact_sel = ((q64 - t64[idx]) ** 2).sum(1)           # exact d^2 of the GPU's choice
    tol = L2_REL * (qn + tn.max())
    assert np.all(exact_sel <= rd.astype(np.float64) ** 2 + 2 * tol)
    np.testing.assert_allclose(d.astype(np.float64) ** 2, exact_sel, rtol=0, atol=float(tol.max()) * 2)
    same = idx == ri
    assert same.mean() > 0.999
    if len(t) > 1:
        exact2 = ((q64 - t64[idx2]) ** 2).sum(1)
        assert np.all(exact2 <= rd2.astype(np.float64) ** 2 + 2 * tol)
        assert np.all(idx2 != idx)
    return same.mean()


def test_l2_golden(gpu, oracle):
    g = np.load(GOLDEN / "matchers.npz")
    idx, d, _, _ = opencv.matchL2(g["lq"], g["lt"])
    np.testing.assert_array_equal(idx, g["l_idx"])
    qn = (g["lq"].astype(np.float64) ** 2).sum(1)
    tn = (g["lt"].astype(np.float64) ** 2).sum(1).max()
    np.testing.assert_array_less(np.abs(d.astype(np.float64) ** 2 - g["l_dist"] ** 2), 2 * L2_REL * (qn + tn))


@pytest.mark.parametrize("nq,nt,dim", [(1, 1, 128), (1, 2, 128), (33, 31, 128), (200, 777, 128), (129, 4099, 128),
                                       (300, 500, 64), (100, 300, 32), (100, 300, 17), (64, 200, 256),
                                       (250, 333, 61)])
def test_l2_shapes(gpu, oracle, nq, nt, dim):
    q, t, _ = S.l2_problem(nq, nt, dim=dim, seed=nq + nt + dim)
    check_l2(oracle, q, t)


def test_l2_ties_lowest_index(gpu):
    rng = np.random.default_rng(3)
    base = S.sift_like(40, 128, rng)
    t = np.concatenate([base, base])
    q = base[rng.integers(0, 40, size=300)]
    idx, d, idx2, d2 = opencv.matchL2(q, t)
    assert (idx < 40).all() and (idx2 == idx + 40).all()
    assert (d < 1.0).all()


def test_l2_medium_vs_oracle(gpu, oracle):
    q, t, planted = S.l2_problem(4000, 6000, dim=128, seed=5)
    frac = check_l2(oracle, q, t)
    idx = opencv.matchL2(q, t)[0]
    ok = planted >= 0
    assert np.mean(idx[ok] == planted[ok]) > 0.99 and frac > 0.999
