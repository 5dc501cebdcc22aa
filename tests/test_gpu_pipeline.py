"""GPU tests of the device-resident match -> RANSAC hand-off (SURVEY §8f row f3:
cvMatchFeatures / cvMatchAndFindModel over the reference's DetectorResult layout).
Bar: the pair list equals the oracle matcher + the stated filters (bit-exact for Hamming), and the
model / mask equal cvFindHomography's (oracle) on the gathered keypoints (mask exact, H 1e-6)."""
import numpy as np
import pytest

from minicv_amd import native as N
from minicv_amd import opencv, synthetic as S

pytestmark = pytest.mark.gpu


def expected_pairs(oracle, da, db, ratio, cross, maxd):
    idx, d1, idx2, d2 = oracle.match_hamming(da, db)
    d1f = d1.astype(np.float32)
    d2f = np.where(d2 == np.iinfo(np.int32).max, np.float32(np.inf), d2.astype(np.float32))
    keep = idx >= 0
    if ratio > 0:
        keep &= d1f < np.float32(ratio) * d2f
    if maxd > 0:
        keep &= d1f <= np.float32(maxd)
    if cross:
        back = oracle.match_hamming(db, da)[0]
        keep &= back[np.maximum(idx, 0)] == np.arange(len(idx))
    q = np.nonzero(keep)[0]
    return np.stack([q, idx[q]], axis=1).astype(np.int32), d1f[q]


def reproj_px(H, pts):
    """median distance (px) between H(pts) and the true H_PIX(pts)"""
    return float(np.median(np.linalg.norm(S.project(H, pts) - S.project(S.H_PIX, pts), axis=1)))


@pytest.mark.parametrize("na,nb,ratio,cross,maxd", [(1000, 1200, 0.8, False, 0), (3000, 2500, 0.75, True, 0),
                                                    (777, 333, 0.0, True, 60.0), (5000, 5000, 0.9, False, 40.0)])
def test_match_features_hamming_exact(gpu, oracle, na, nb, ratio, cross, maxd):
    pa, da, pb, db, planted = S.feature_pair_problem(na, nb, seed=na + nb)
    A, B = opencv.Features(pa, da), opencv.Features(pb, db)
    pairs, dist = opencv.matchFeatures(A, B, ratio=ratio, cross_check=cross, max_distance=maxd)
    ep, ed = expected_pairs(oracle, da, db, ratio, cross, maxd)
    np.testing.assert_array_equal(pairs, ep)
    np.testing.assert_array_equal(dist, ed)


def test_match_and_find_homography_vs_oracle(gpu, oracle):
    pa, da, pb, db, planted = S.feature_pair_problem(4000, 4000, seed=21, match_frac=0.5)
    A, B = opencv.Features(pa, da), opencv.Features(pb, db)
    p = opencv.RansacParams(threshold=3.0, confidence=0.995, max_iters=2000, seed=5)
    cnt, H, pairs, mask = opencv.matchAndFindModel(A, B, ratio=0.8, cross_check=True, params=p)
    ep, _ = expected_pairs(oracle, da, db, 0.8, True, 0)
    np.testing.assert_array_equal(pairs, ep)
    src = pa[ep[:, 0]].astype(np.float32).astype(np.float64)
    dst = pb[ep[:, 1]].astype(np.float32).astype(np.float64)
    rc, rH, rmask, _ = oracle.find_homography(src, dst, thr=3.0, conf=0.995, max_iters=2000, seed=5)
    assert cnt == rc
    np.testing.assert_array_equal(mask, rmask != 0)
    Hn, rHn = H / np.linalg.norm(H), rH / np.linalg.norm(rH)
    assert np.linalg.norm(Hn - rHn) < 1e-6
    assert reproj_px(H, pa) < 0.5
    # every inlier is a planted correspondence
    assert (planted[pairs[mask, 0]] == pairs[mask, 1]).mean() > 0.99


def test_match_and_find_fundamental(gpu, oracle):
    pa, da, pb, db, planted = S.feature_pair_problem(3000, 3000, seed=22, match_frac=0.6)
    A, B = opencv.Features(pa, da), opencv.Features(pb, db)
    p = opencv.RansacParams(threshold=2.0, confidence=0.99, max_iters=1000, seed=3)
    cnt, F, pairs, mask = opencv.matchAndFindModel(A, B, model=N.MODEL_FUNDAMENTAL, ratio=0.8, params=p)
    ep, _ = expected_pairs(oracle, da, db, 0.8, False, 0)
    np.testing.assert_array_equal(pairs, ep)
    src = pa[ep[:, 0]].astype(np.float32).astype(np.float64)
    dst = pb[ep[:, 1]].astype(np.float32).astype(np.float64)
    rc, rF, rmask, _ = oracle.find_fundamental(src, dst, thr=2.0, conf=0.99, max_iters=1000, seed=3)
    assert cnt == rc
    np.testing.assert_array_equal(mask, rmask != 0)
    np.testing.assert_array_equal(F, rF)


def test_match_features_l2(gpu):
    pa, da, pb, db, planted = S.feature_pair_problem(2000, 2500, seed=23, kind="l2", match_frac=0.7)
    A, B = opencv.Features(pa, da), opencv.Features(pb, db)
    pairs, dist = opencv.matchFeatures(A, B, ratio=0.8, cross_check=True)
    ok = planted[pairs[:, 0]] >= 0
    assert ok.mean() > 0.95 and (planted[pairs[ok, 0]] == pairs[ok, 1]).mean() > 0.99
    assert np.all(np.diff(pairs[:, 0]) > 0)
    cnt, H, pr, mask = opencv.matchAndFindModel(A, B, ratio=0.8, cross_check=True,
                                                params=opencv.RansacParams(threshold=3.0, seed=1))
    assert reproj_px(H, pa) < 0.5


def test_pipeline_edge_cases(gpu):
    pa, da, pb, db, _ = S.feature_pair_problem(100, 100, seed=24)
    A = opencv.Features(pa, da)
    empty = opencv.Features(np.zeros((0, 2)), np.zeros((0, 32), np.uint8))
    pairs, dist = opencv.matchFeatures(A, empty)
    assert len(pairs) == 0
    with pytest.raises(N.NativeError, match="element types differ"):
        opencv.matchFeatures(A, opencv.Features(pb, db.astype(np.float32)))
    with pytest.raises(N.NativeError, match="need at least"):
        opencv.matchAndFindModel(opencv.Features(pa[:3], da[:3]), opencv.Features(pb, db), ratio=0.0)
