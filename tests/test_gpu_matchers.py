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
