"""GPU parity of the essential-matrix path behind the reference's own exports
cvRecoverPose / cvRecoverPoses / cvFivePoint (MiniCVNative.cpp:165-215, 368-382) and the new
cvFindEssentialMat, against the oracle (oracle/oracle_e.c).
Bar: five-point models, per-slot inlier counts, masks and the returned E bit-exact; the pose from
recoverPose (R, t, cheirality count) bit-exact; plus geometric truth on synthetic two-view data."""
import ctypes as C

import numpy as np
import pytest

from minicv_amd import native as N
from minicv_amd import opencv, synthetic as S

pytestmark = pytest.mark.gpu

FOCAL, PP = 800.0, (640.0, 360.0)


@pytest.fixture(scope="module")
def torch_dev(gpu):
    import torch
    return torch, torch.device("cuda:0")


def test_five_point_bit_exact(gpu, oracle):
    rng = np.random.default_rng(3)
    for trial in range(60):
        if trial % 3 == 0:
            a, b = rng.normal(size=(5, 2)), rng.normal(size=(5, 2))
        else:
            a, b, *_ = S.essential_problem(5, seed=trial, outlier_frac=0, sigma=0.0 if trial % 2 else 0.4,
                                           focal=1.0, pp=(0, 0))
        Es = opencv.fivepoint(a, b)
        ref = oracle.e_solve5_ref(a[:, 0], a[:, 1], b[:, 0], b[:, 1])   # the export's own path
        assert len(Es) == len(ref)
        for e, r in zip(Es, ref):
            np.testing.assert_array_equal(e, r)


def test_five_point_exact_geometry(gpu):
    a, b, _, R, tu, E = S.essential_problem(5, seed=21, outlier_frac=0, sigma=0, focal=1.0, pp=(0, 0))
    Es = opencv.fivepoint(a, b)
    assert min(min(np.abs(e - E).max(), np.abs(e + E).max()) for e in Es) < 1e-8


@pytest.mark.parametrize("n,outl,seed,begin,count,unfused,fast", [
    (5, 0.0, 1, 0, 64, False, False), (6, 0.3, 2, 0, 100, False, False), (300, 0.5, 3, 0, 512, False, False),
    (2000, 0.5, 4, 123457, 512, False, False), (1999, 0.6, 5, 0, 256, True, False),
    (64, 0.2, 6, 2**28, 300, False, False), (1000, 0.5, 11, 5, 20000, True, False),
    (300, 0.5, 8, 77, 50000, False, False), (5, 0.0, 10, 0, 32768, False, False),
    # MCV_FLAG_FAST_MINIMAL (the replacement solver); >= kEStageMinHyps hypotheses per chunk take its
    # split path (matrix phases per 16-lane group, roots per 4-lane group)
    (300, 0.5, 3, 0, 512, False, True), (1000, 0.5, 12, 5, 33000, True, True), (5, 0.0, 10, 0, 32768, False, True)])
def test_e_slot_counts_bit_exact(torch_dev, oracle, n, outl, seed, begin, count, unfused, fast):
    torch, dev = torch_dev
    from minicv_amd import device as D
    a, b, *_ = S.essential_problem(n, seed=seed, outlier_frac=outl)
    pts = D.pack_essential_tensor(a, b, FOCAL, PP, dev)
    ref_pts = oracle.pack_e(a, b, FOCAL, PP)
    np.testing.assert_array_equal(pts.cpu().numpy(), ref_pts)          # normalisation on the GPU
    plan = D.RansacPlan(N.MODEL_ESSENTIAL, n, count)
    thr = 1.0 / FOCAL                                                  # device API: normalised units
    cfg = opencv.RansacParams(threshold=thr, seed=seed, fused_error=not unfused, fast_minimal=fast).to_c()
    key = torch.zeros(2, dtype=torch.int64, device=dev)
    counts = torch.zeros(count * N.E_SLOTS, dtype=torch.int32, device=dev)
    plan.evaluate(pts, n, cfg, begin, count, key, counts)
    got = counts.cpu().numpy()
    with oracle.fast_minimal(fast):
        ref = oracle.e_counts(ref_pts, seed, begin, count, float(np.float32(thr * thr)), 1 if unfused else 0)
    np.testing.assert_array_equal(got, ref)
    if (ref >= 5).any() and not (ref == -2).any():
        c = ref.max()
        i = int(np.nonzero(ref == c)[0][0])
        assert int(key[0].item()) == (int(c) << 32) | (0xFFFFFFFF - (begin * N.E_SLOTS + i))
    plan.close()


@pytest.mark.parametrize("n,outl,seed,iters,conf,flags", [
    (6, 0.0, 1, 1000, 0.999, 0), (50, 0.3, 2, 1000, 0.999, 0), (500, 0.5, 3, 1000, 0.999, 0),
    (3000, 0.5, 4, 1000, 0.999, 0), (3000, 0.6, 5, 300, 0.999, N.FLAG_FIXED_ITERS),
    (2000, 0.5, 6, 1000, 0.99, N.FLAG_FUSED_ERROR), (20000, 0.5, 7, 1000, 0.999, 0),
    (3000, 0.5, 4, 1000, 0.999, N.FLAG_FAST_MINIMAL), (3000, 0.5, 8, 1000, 0.999, N.FLAG_CV_SAMPLER)])
def test_find_essential_vs_oracle(gpu, oracle, n, outl, seed, iters, conf, flags):
    a, b, inl, R, tu, E = S.essential_problem(n, seed=seed, outlier_frac=outl)
    p = opencv.RansacParams(threshold=1.0, confidence=conf, max_iters=iters, seed=seed,
                            fixed_iters=bool(flags & N.FLAG_FIXED_ITERS),
                            fused_error=bool(flags & N.FLAG_FUSED_ERROR),
                            fast_minimal=bool(flags & N.FLAG_FAST_MINIMAL), cv_sampler=bool(flags & N.FLAG_CV_SAMPLER))
    cnt, Eg, mask = opencv.findEssentialMat(a, b, FOCAL, PP, p)
    rc, Er, rmask, best = oracle.find_essential(a, b, FOCAL, PP, thr=1.0, conf=conf, max_iters=iters, seed=seed,
                                                flags=flags)
    assert cnt == rc
    np.testing.assert_array_equal(Eg, Er)
    np.testing.assert_array_equal(mask, rmask != 0)
    if n >= 500:
        assert min(np.abs(Eg - E).max(), np.abs(Eg + E).max()) < 0.15   # best minimal-sample model, no refit


def test_find_essential_n5(gpu, oracle):
    for seed in range(12):
        a, b, *_ = S.essential_problem(5, seed=seed, outlier_frac=0)
        ref = oracle.find_essential(a, b, FOCAL, PP)
        if ref[0] == 5:
            cnt, Eg, mask = opencv.findEssentialMat(a, b, FOCAL, PP)
            assert cnt == 5 and mask.all()
            np.testing.assert_array_equal(Eg, ref[1])
        else:
            with pytest.raises(N.NativeError, match="solutions"):
                opencv.findEssentialMat(a, b, FOCAL, PP)


@pytest.mark.parametrize("n,outl,seed,thr", [(200, 0.3, 1, 0.5), (5000, 0.5, 2, 1.0), (30000, 0.4, 3, 2.0)])
def test_recover_pose_vs_oracle(gpu, oracle, n, outl, seed, thr):
    a, b, inl, R, tu, E = S.essential_problem(n, seed=seed, outlier_frac=outl, sigma=0.2)
    cfg = opencv.recoverPoseConfig(FOCAL, PP, 0.999, thr)
    res, Rg, tg, ms = opencv.recoverPose(cfg, a, b)
    rc, Er, rmask, _ = oracle.find_essential(a, b, FOCAL, PP, thr=thr, conf=0.999, max_iters=1000,
                                             flags=N.FLAG_CV_SAMPLER)   # OpenCV's own sample stream
    np.testing.assert_array_equal(ms, rmask)                          # ms = RANSAC mask (:206-210)
    rres, Rr, tr, g = oracle.recover_pose(a, b, Er, rmask, FOCAL, PP)
    assert res == rres
    np.testing.assert_array_equal(Rg, Rr)
    np.testing.assert_array_equal(tg, tr)
    assert np.abs(Rg - R).max() < 0.03 and np.abs(tg - tu).max() < 0.08
    assert res > 0.9 * ms.sum()


def test_recover_poses_vs_oracle(gpu, oracle):
    a, b, inl, R, tu, E = S.essential_problem(4000, seed=9, outlier_frac=0.5, sigma=0.2)
    cfg = opencv.recoverPoseConfig(FOCAL, PP, 0.999, 1.0)
    R1, R2, t, ms = opencv.recoverPoses(cfg, a, b)
    rc, Er, rmask, _ = oracle.find_essential(a, b, FOCAL, PP, thr=1.0, conf=0.999, max_iters=1000,
                                             flags=N.FLAG_CV_SAMPLER)
    np.testing.assert_array_equal(ms, rmask)
    oR1, oR2, ot = oracle.e_decompose(Er)
    np.testing.assert_array_equal(R1, oR1)
    np.testing.assert_array_equal(R2, oR2)
    np.testing.assert_array_equal(t, ot)
    assert min(np.abs(R1 - R).max(), np.abs(R2 - R).max()) < 0.03


def test_recover_poses2_convention(gpu):
    # NDC-like input of OpenCV.fs:872-909: (x, y) in [-1, 1], y up
    a, b, inl, R, tu, E = S.essential_problem(2000, seed=4, outlier_frac=0.3, sigma=0.1, focal=400.0, pp=(0, 0))
    poses, mask = opencv.recoverPoses2(opencv.recoverPoseConfig(1.0, (0, 0), 0.999, 1.0 / 400.0), a / 400.0,
                                       b / 400.0)
    assert 1 <= len(poses) <= 2 and mask.sum() > 0.8 * inl.sum()


def test_recover_edge_cases(gpu, oracle):
    cfg = opencv.recoverPoseConfig(FOCAL, PP, 0.999, 1.0)
    a, b, *_ = S.essential_problem(4, seed=1, outlier_frac=0)
    R1, R2, t, ms = opencv.recoverPoses(cfg, a, b)                     # N < 5: false, outputs untouched
    np.testing.assert_array_equal(R1, np.eye(3))
    assert list(t) == [100, 123, 432] and not ms.any()
    with pytest.raises(N.NativeError, match="at least 5"):
        opencv.recoverPose(cfg, a, b)
    # all points identical: every sample is degenerate. fivepoint.cpp's arithmetic still returns
    # models there (the SVD null space of a rank-1 system is some 4-dimensional basis, and the
    # polynomial has real roots), every point is an inlier of them, and the pose follows — the
    # product must return what the restated reference returns
    a = np.tile([[100.0, 200.0]], (50, 1))
    b = np.tile([[110.0, 190.0]], (50, 1))
    R1, R2, t, ms = opencv.recoverPoses(cfg, a, b)
    rc, Er, rmask, _ = oracle.find_essential(a, b, FOCAL, PP, thr=1.0, conf=0.999, max_iters=1000,
                                             flags=N.FLAG_CV_SAMPLER)
    assert rc == 50
    np.testing.assert_array_equal(ms, rmask)
    oR1, oR2, ot = oracle.e_decompose(Er)
    np.testing.assert_array_equal(t, ot)
    # the replacement solver (opt-in) finds no model on the degenerate set, on both sides
    rc_f, *_ = oracle.find_essential(a, b, FOCAL, PP, thr=1.0, conf=0.999, max_iters=1000,
                                     flags=N.FLAG_CV_SAMPLER | N.FLAG_FAST_MINIMAL)
    assert rc_f == 0
    fp = opencv.RansacParams(threshold=1.0, confidence=0.999, max_iters=1000, cv_sampler=True, fast_minimal=True)
    with pytest.raises(N.NativeError, match="no model"):
        opencv.findEssentialMat(a, b, FOCAL, PP, fp)
    with pytest.raises(N.NativeError, match="confidence"):
        opencv.recoverPose(opencv.recoverPoseConfig(FOCAL, PP, 1.5, 1.0), *S.essential_problem(50, seed=2)[:2])


def test_raw_export_marshalling(native, gpu):
    """cvRecoverPose through ctypes exactly like the F# P/Invoke (OpenCV.fs:855-861)."""
    a, b, *_ = S.essential_problem(500, seed=12, outlier_frac=0.2)
    cfg = N.RecoverPoseConfig(FOCAL, N.V2d(*PP), 0.999, 1.0)
    m, t = N.M33d(), N.V3d(100, 123, 432)
    ms = np.zeros(500, np.uint8)
    pa, pb = np.ascontiguousarray(a), np.ascontiguousarray(b)
    res = native.lib().cvRecoverPose(C.addressof(cfg), 500, pa.ctypes.data, pb.ctypes.data, C.addressof(m),
                                     C.addressof(t), ms.ctypes.data)
    assert res > 300 and set(np.unique(ms)) <= {0, 1}
    Rm = np.array(m.M[:]).reshape(3, 3)
    np.testing.assert_allclose(Rm @ Rm.T, np.eye(3), atol=1e-12)


def test_e_counts_at_exact_threshold_boundary(torch_dev, oracle):
    torch, dev = torch_dev
    from minicv_amd import device as D
    from test_gpu_fundamental import _sampson_unfused_np, _thr_for
    a, b, *_ = S.essential_problem(3000, seed=13, outlier_frac=0.3)
    p = oracle.pack_e(a, b, FOCAL, PP)
    n0, E90, _ = oracle.e_hypothesis(p, 13, 0)
    assert n0 >= 1
    x = p.astype(np.float64)
    F = E90[0]
    ax = F[0] * x[:, 0] + F[1] * x[:, 1] + F[2] * 1.0
    ay = F[3] * x[:, 0] + F[4] * x[:, 1] + F[5] * 1.0
    az = F[6] * x[:, 0] + F[7] * x[:, 1] + F[8] * 1.0
    bx = F[0] * x[:, 2] + F[3] * x[:, 3] + F[6] * 1.0
    by = F[1] * x[:, 2] + F[4] * x[:, 3] + F[7] * 1.0
    c = x[:, 2] * ax + x[:, 3] * ay + 1.0 * az
    err = (c * c / (ax * ax + ay * ay + bx * bx + by * by)).astype(np.float32)
    pts = D.pack_essential_tensor(a, b, FOCAL, PP, dev)
    plan = D.RansacPlan(N.MODEL_ESSENTIAL, 3000, 32)
    for q in (0.2, 0.6):
        target = np.float32(np.quantile(err, q, method="nearest"))
        thr = _thr_for(target)
        for unfused in (True, False):
            cfg = opencv.RansacParams(threshold=thr, seed=13, fused_error=not unfused).to_c()
            key = torch.zeros(2, dtype=torch.int64, device=dev)
            counts = torch.zeros(32 * N.E_SLOTS, dtype=torch.int32, device=dev)
            plan.evaluate(pts, 3000, cfg, 0, 32, key, counts)
            ref = oracle.e_counts(p, 13, 0, 32, float(target), 1 if unfused else 0)
            np.testing.assert_array_equal(counts.cpu().numpy(), ref)
            if unfused:
                assert ref[0] == int((err <= target).sum())
    plan.close()


@pytest.mark.parametrize("case", ["nan", "wide_thr"])
def test_e_counts_prefilter_extremes(torch_dev, oracle, case):
    """E sweep through the packed-fp32 prefilter: a NaN coordinate (no certification at all) and a
    threshold wide enough to put many correspondences near the cut; bit-exact against the oracle."""
    torch, dev = torch_dev
    from minicv_amd import device as D
    n, count, seed = 1200, 128, 23
    a, b, *_ = S.essential_problem(n, seed=seed, outlier_frac=0.4)
    a, b = a.copy(), b.copy()
    thr = 1.0 / FOCAL
    if case == "nan":
        b[7, 1] = np.nan
    else:
        thr = 20.0 / FOCAL
    pts = D.pack_essential_tensor(a, b, FOCAL, PP, dev)
    ref_pts = oracle.pack_e(a, b, FOCAL, PP)
    plan = D.RansacPlan(N.MODEL_ESSENTIAL, n, count)
    for unfused in (False, True):
        cfg = opencv.RansacParams(threshold=thr, seed=seed, fused_error=not unfused).to_c()
        key = torch.zeros(2, dtype=torch.int64, device=dev)
        counts = torch.zeros(count * N.E_SLOTS, dtype=torch.int32, device=dev)
        plan.evaluate(pts, n, cfg, 0, count, key, counts)
        ref = oracle.e_counts(ref_pts, seed, 0, count, float(np.float32(thr * thr)), 1 if unfused else 0)
        np.testing.assert_array_equal(counts.cpu().numpy(), ref)
        assert (ref > 0).any()
    plan.close()


@pytest.mark.slow
def test_e_counts_bench_workload_full(torch_dev, oracle):
    """bench.py's essential workload at full size (100k correspondences, 2^20 hypotheses in one
    evaluate, <= 10 model slots each): every slot's status / count in a 262144-hypothesis sample over
    the whole range (every 8-rank share's first and last 1024, 240 strided blocks, the bench's reported
    winner, slot 1,451,982 = hypothesis 145,198, and the device's argmax) equals the oracle's."""
    import _sample
    torch, dev = torch_dev
    from minicv_amd import device as D
    n, H, focal, pp = 100_000, 1 << 20, 800.0, (640.0, 360.0)
    a, b, *_ = S.essential_problem(n, seed=6, outlier_frac=0.5)
    pts = D.pack_essential_tensor(a, b, focal, pp, dev)
    plan = D.RansacPlan(N.MODEL_ESSENTIAL, n, H)
    thr = 1.0 / focal
    cfg = opencv.RansacParams(threshold=thr, seed=6, fixed_iters=True, max_iters=H).to_c()
    key = torch.zeros(2, dtype=torch.int64, device=dev)
    counts = torch.zeros(H * N.E_SLOTS, dtype=torch.int32, device=dev)
    plan.evaluate(pts, n, cfg, 0, H, key, counts)
    c = counts.cpu().numpy()
    cnt, slot = D.unpack_key(int(key[0].item()))
    assert cnt == c.max() and slot == int(np.argmax(c))
    assert slot == 1_451_982, "bench.py's reported essential winner (profiles/r04_bench_essential.json)"
    pe = oracle.pack_e(a, b, focal, pp)
    thr2 = float(np.float32(thr * thr))
    ranges = _sample.bench_sample(H, around=(slot // N.E_SLOTS,))
    print("essential sample:", _sample.describe(ranges))
    S_ = N.E_SLOTS
    for lo, hi in ranges:
        np.testing.assert_array_equal(c[lo * S_:hi * S_], oracle.e_counts(pe, 6, lo, hi - lo, thr2, 1),
                                      err_msg=f"[{lo},{hi})")
    plan.close()
