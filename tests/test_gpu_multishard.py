"""RansacConfig.deviceCount > 1 on the host-pointer exports: every chunk of hypotheses is split over
per-shard workspaces (round-robin over the visible GPUs; on a one-GPU box the shards share it)
and the counts are replayed in order — the result must be bit-identical to deviceCount = 1."""
import numpy as np
import pytest

from minicv_amd import native as N
from minicv_amd import opencv, synthetic as S

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shards", [2, 3, 8])
@pytest.mark.parametrize("fixed", [False, True])
def test_homography_shards_identical(gpu, shards, fixed):
    src, dst, _ = S.homography_problem(5000, 7, outlier_frac=0.6)
    base = opencv.RansacParams(threshold=5e-3, seed=11, max_iters=3000, fixed_iters=fixed)
    multi = opencv.RansacParams(threshold=5e-3, seed=11, max_iters=3000, fixed_iters=fixed, device_count=shards)
    c1, H1, m1 = opencv.findHomography(src, dst, base)
    c2, H2, m2 = opencv.findHomography(src, dst, multi)
    assert c1 == c2
    np.testing.assert_array_equal(H1, H2)
    np.testing.assert_array_equal(m1, m2)


@pytest.mark.parametrize("shards", [2, 5])
@pytest.mark.parametrize("fixed", [False, True])
def test_fundamental_essential_pnp_shards_identical(gpu, shards, fixed):
    """fixed = True: each shard reduces its range to a 16-byte key on its device (no count gather)."""
    a, b, _, _ = S.fundamental_problem(4000, 8, outlier_frac=0.5)
    p1 = opencv.RansacParams(threshold=5e-3, confidence=0.99, seed=3, max_iters=2000, fixed_iters=fixed)
    pk = opencv.RansacParams(threshold=5e-3, confidence=0.99, seed=3, max_iters=2000, device_count=shards,
                             fixed_iters=fixed)
    r1, r2 = opencv.findFundamentalMat(a, b, p1), opencv.findFundamentalMat(a, b, pk)
    assert r1[0] == r2[0]
    np.testing.assert_array_equal(r1[1], r2[1])
    np.testing.assert_array_equal(r1[2], r2[2])

    a, b, *_ = S.essential_problem(3000, seed=9, outlier_frac=0.5)
    e1 = opencv.RansacParams(threshold=1.0, confidence=0.999, seed=4, max_iters=1000, fixed_iters=fixed)
    ek = opencv.RansacParams(threshold=1.0, confidence=0.999, seed=4, max_iters=1000, device_count=shards,
                             fixed_iters=fixed)
    r1 = opencv.findEssentialMat(a, b, 800.0, (640.0, 360.0), e1)
    r2 = opencv.findEssentialMat(a, b, 800.0, (640.0, 360.0), ek)
    assert r1[0] == r2[0]
    np.testing.assert_array_equal(r1[1], r2[1])
    np.testing.assert_array_equal(r1[2], r2[2])

    img, W, inl, K, d, R, t = S.pnp_problem(3000, seed=10, outlier_frac=0.5, dist=[-0.1, 0.02, 0.001, 0.0])
    q1 = opencv.RansacParams(threshold=2.0, confidence=0.99, seed=5, max_iters=300, fixed_iters=fixed)
    qk = opencv.RansacParams(threshold=2.0, confidence=0.99, seed=5, max_iters=300, device_count=shards,
                             fixed_iters=fixed)
    s1 = opencv.solvePnPRansac(img, W, K, d, params=q1)
    s2 = opencv.solvePnPRansac(img, W, K, d, params=qk)
    assert s1[0] and s2[0]
    for x, y in zip(s1[1:], s2[1:]):
        np.testing.assert_array_equal(x, y)


def test_fixed_shards_with_sampler_failure(gpu, oracle):
    """A point set whose every homography sample is rejected: getSubset fails at hypothesis 0, the
    fixed-iteration key path sees the failure and falls back to the in-order replay (no model)."""
    n = 60
    t = np.linspace(-1, 1, n)
    src = np.stack([t, t], 1)
    dst = np.stack([t, -t], 1)
    for shards in (1, 3):
        p = opencv.RansacParams(threshold=5e-3, seed=2, max_iters=500, fixed_iters=True, device_count=shards)
        with pytest.raises(N.NativeError, match="no model"):
            opencv.findHomography(src, dst, p)
