"""GPU parity of the fundamental-matrix RANSAC path (8-point minimal sets) against the oracle.
Bar: per-hypothesis inlier counts and masks bit-exact for all four error definitions; the returned
F (best hypothesis' fp64 model, no refit — as OpenCV's findFundamentalMat) bit-identical; the
all-points 8-point fit within 1e-6 relative Frobenius (GPU fp64 sums in another order)."""
import numpy as np
import pytest

from minicv_amd import native as N
from minicv_amd import opencv, synthetic as S

pytestmark = pytest.mark.gpu


def relf_up_to_sign(A, B):
    A = A / np.linalg.norm(A)
    B = B / np.linalg.norm(B)
    return min(np.linalg.norm(A - B), np.linalg.norm(A + B))


@pytest.fixture(scope="module")
def torch_dev(gpu):
    import torch
    return torch, torch.device("cuda:0")


@pytest.mark.parametrize("n,outl,seed,begin,count,error_kind,unfused", [
    (8, 0.0, 1, 0, 64, 0, False), (9, 0.3, 2, 0, 200, 0, False), (300, 0.5, 3, 0, 1024, 0, False),
    (2000, 0.5, 4, 77777, 1024, 0, False), (1999, 0.5, 5, 0, 512, 0, True), (1000, 0.6, 6, 0, 512, 1, False),
    (1000, 0.6, 7, 2**31, 512, 1, True), (65, 0.2, 8, 0, 300, 1, False)])
def test_f_counts_bit_exact(torch_dev, oracle, n, outl, seed, begin, count, error_kind, unfused):
    torch, dev = torch_dev
    from minicv_amd import device as D
    a, b, _, _ = S.fundamental_problem(n, seed, outlier_frac=outl)
    pts = D.pack_points_tensor(a, b, dev)
    plan = D.RansacPlan(N.MODEL_FUNDAMENTAL, n, count)
    thr = 5e-3
    cfg = opencv.RansacParams(threshold=thr, seed=seed, error_kind=error_kind, fused_error=not unfused).to_c()
    key = torch.zeros(2, dtype=torch.int64, device=dev)
    counts = torch.zeros(count, dtype=torch.int32, device=dev)
    plan.evaluate(pts, n, cfg, begin, count, key, counts)
    got = counts.cpu().numpy()
    ref = oracle.f_counts(oracle.pack4(a, b), seed, begin, count, float(np.float32(thr * thr)),
                          oracle.f_kind(error_kind, unfused))
    np.testing.assert_array_equal(got, ref)
    valid = ref >= 8
    k = int(key[0].item())
    if valid.any() and not (ref == -2).any():
        c = ref.max()
        i = int(np.nonzero(ref == c)[0][0])
        assert k == (int(c) << 32) | (0xFFFFFFFF - (begin + i))
    plan.close()


@pytest.mark.parametrize("n,outl,seed,begin,count", [(8, 0.0, 31, 0, 64), (2000, 0.5, 32, 5, 1024)])
def test_f_counts_fast_minimal(torch_dev, oracle, n, outl, seed, begin, count):
    """MCV_FLAG_FAST_MINIMAL (elimination null vector) against the oracle's elimination."""
    torch, dev = torch_dev
    from minicv_amd import device as D
    a, b, _, _ = S.fundamental_problem(n, seed, outlier_frac=outl)
    pts = D.pack_points_tensor(a, b, dev)
    plan = D.RansacPlan(N.MODEL_FUNDAMENTAL, n, count)
    thr = 5e-3
    cfg = opencv.RansacParams(threshold=thr, seed=seed, fast_minimal=True).to_c()
    key = torch.zeros(2, dtype=torch.int64, device=dev)
    counts = torch.zeros(count, dtype=torch.int32, device=dev)
    plan.evaluate(pts, n, cfg, begin, count, key, counts)
    got = counts.cpu().numpy()
    with oracle.fast_minimal():
        ref = oracle.f_counts(oracle.pack4(a, b), seed, begin, count, float(np.float32(thr * thr)),
                              oracle.f_kind(0, True))
    np.testing.assert_array_equal(got, ref)
    plan.close()
    if n == 8:
        return   # N == 8 is one all-points fit (GPU sums, 1e-6 bar: test_find_fundamental_vs_oracle)
    with oracle.fast_minimal():
        cnt_o, F_o, mask_o, _ = oracle.find_fundamental(a, b, thr=thr, seed=seed, max_iters=300)
    cnt, F, mask = opencv.findFundamentalMat(a, b, opencv.RansacParams(threshold=thr, seed=seed, max_iters=300,
                                                                       confidence=0.99, fast_minimal=True))
    assert cnt == cnt_o
    np.testing.assert_array_equal(mask, mask_o.astype(bool))
    np.testing.assert_array_equal(F, F_o)


@pytest.mark.parametrize("n,outl,seed,iters,conf,error_kind,flags", [
    (8, 0.0, 1, 1000, 0.99, 0, 0), (50, 0.3, 2, 1000, 0.99, 0, 0), (500, 0.5, 4, 1000, 0.99, 0, 0),
    (3000, 0.5, 5, 2000, 0.99, 0, 0), (3000, 0.5, 6, 2000, 0.99, 1, 0),
    (2000, 0.5, 7, 500, 0.99, 0, N.FLAG_FIXED_ITERS), (2000, 0.5, 8, 1000, 0.999, 1, N.FLAG_FUSED_ERROR)])
def test_find_fundamental_vs_oracle(gpu, oracle, n, outl, seed, iters, conf, error_kind, flags):
    a, b, _, _ = S.fundamental_problem(n, seed, outlier_frac=outl)
    thr = 5e-3
    cnt_o, F_o, mask_o, _ = oracle.find_fundamental(a, b, thr=thr, conf=conf, max_iters=iters, seed=seed,
                                                    flags=flags, error_kind=error_kind)
    p = opencv.RansacParams(threshold=thr, confidence=conf, max_iters=iters, seed=seed, error_kind=error_kind,
                            fixed_iters=bool(flags & N.FLAG_FIXED_ITERS),
                            fused_error=bool(flags & N.FLAG_FUSED_ERROR))
    cnt, F, mask = opencv.findFundamentalMat(a, b, p)
    assert cnt == cnt_o
    np.testing.assert_array_equal(mask, mask_o.astype(bool))
    if n == 8:
        assert relf_up_to_sign(F, F_o) < 1e-6   # all-points fit path
    else:
        np.testing.assert_array_equal(F, F_o)


def test_fundamental_lsq(gpu, oracle):
    a, b, inl, Ft = S.fundamental_problem(4000, 9, outlier_frac=0.0)
    cnt_o, F_o, _, _ = oracle.find_fundamental(a, b, method=0)
    cnt, F, mask = opencv.findFundamentalMat(a, b, opencv.RansacParams(method=N.METHOD_LSQ))
    assert cnt == cnt_o == 4000 and mask.all()
    assert relf_up_to_sign(F, F_o) < 1e-6


def test_fundamental_golden(gpu):
    from pathlib import Path
    g = np.load(Path(__file__).resolve().parent / "golden" / "fundamental.npz")
    p = opencv.RansacParams(threshold=float(g["thr"]), confidence=float(g["conf"]), max_iters=int(g["max_iters"]),
                            seed=int(g["seed"]))
    cnt, F, mask = opencv.findFundamentalMat(g["a"], g["b"], p)
    assert cnt == int(g["count"])
    np.testing.assert_array_equal(mask, g["mask"].astype(bool))
    np.testing.assert_array_equal(F, g["F"])


def test_fundamental_degenerate(gpu):
    x = np.linspace(-1, 1, 40)
    a = np.stack([x, 0.5 * x], axis=1)
    with pytest.raises(N.NativeError):
        opencv.findFundamentalMat(a, a.copy(), opencv.RansacParams(threshold=0.01))
    with pytest.raises(N.NativeError):
        opencv.findFundamentalMat(a[:7], a[:7])


def _sampson_unfused_np(F, p4):
    """Op-by-op Sampson error exactly as f_err_sampson (numpy float64 has no FMA contraction)."""
    F = np.asarray(F, dtype=np.float64).ravel()
    x1, y1, x2, y2 = (p4[:, k].astype(np.float64) for k in range(4))
    ax = F[0] * x1 + F[1] * y1 + F[2] * 1.0
    ay = F[3] * x1 + F[4] * y1 + F[5] * 1.0
    az = F[6] * x1 + F[7] * y1 + F[8] * 1.0
    bx = F[0] * x2 + F[3] * y2 + F[6] * 1.0
    by = F[1] * x2 + F[4] * y2 + F[7] * 1.0
    c = x2 * ax + y2 * ay + 1.0 * az
    return (c * c / (ax * ax + ay * ay + bx * bx + by * by)).astype(np.float32)


def _thr_for(target: np.float32) -> float:
    """A double thr with (float)(thr * thr) == target."""
    t = float(np.sqrt(np.float64(target)))
    for _ in range(200):
        got = np.float32(t * t)
        if got == target:
            return t
        t = float(np.nextafter(t, np.inf if got < target else -np.inf))
    raise AssertionError("no threshold maps to the target")


@pytest.mark.parametrize("unfused", [True, False])
def test_f_counts_at_exact_threshold_boundary(torch_dev, oracle, unfused):
    """Thresholds equal to actual float errors of many points: the certified division-free compare
    must hand these boundary cases to the exact path (err == thr2 is an inlier)."""
    torch, dev = torch_dev
    from minicv_amd import device as D
    a, b, _, _ = S.fundamental_problem(3000, 12, outlier_frac=0.3)
    p4 = oracle.pack4(a, b)
    st, F, _ = oracle.f_hypothesis(p4, 12, 0)
    assert st == 1
    err = _sampson_unfused_np(F, p4)
    pts = D.pack_points_tensor(a, b, dev)
    plan = D.RansacPlan(N.MODEL_FUNDAMENTAL, 3000, 64)
    for q in (0.1, 0.5, 0.9):
        target = np.float32(np.quantile(err, q, method="nearest"))
        thr = _thr_for(target)
        cfg = opencv.RansacParams(threshold=thr, seed=12, fused_error=not unfused).to_c()
        key = torch.zeros(2, dtype=torch.int64, device=dev)
        counts = torch.zeros(64, dtype=torch.int32, device=dev)
        plan.evaluate(pts, 3000, cfg, 0, 64, key, counts)
        ref = oracle.f_counts(p4, 12, 0, 64, float(target), oracle.f_kind(0, unfused))
        np.testing.assert_array_equal(counts.cpu().numpy(), ref)
        if unfused:
            assert ref[0] == int((err <= target).sum())
    plan.close()


@pytest.mark.parametrize("case", ["nan", "huge", "tiny", "wide_thr"])
def test_f_counts_prefilter_extremes(torch_dev, oracle, case):
    """The packed-fp32 prefilter (sampson_pk.h) against the fp64 oracle where its bound must give
    up: a NaN coordinate (bound -> inf: every lane re-tested in fp64), a 1e30 coordinate (bound out
    of range), a point set scaled by 1e-30 (magnitudes below the bound's range), and a threshold
    wide enough to put many correspondences near the cut."""
    torch, dev = torch_dev
    from minicv_amd import device as D
    n, count, seed = 1500, 256, 21
    a, b, _, _ = S.fundamental_problem(n, seed, outlier_frac=0.4)
    a, b = a.copy(), b.copy()
    thr = 5e-3
    if case == "nan":
        a[10, 0] = np.nan
    elif case == "huge":
        b[20, 0] = 1e30
    elif case == "tiny":
        a *= 1e-30
        b *= 1e-30
        thr = 5e-33
    else:
        thr = 0.5
    pts = D.pack_points_tensor(a, b, dev)
    plan = D.RansacPlan(N.MODEL_FUNDAMENTAL, n, count)
    for unfused in (False, True):
        cfg = opencv.RansacParams(threshold=thr, seed=seed, fused_error=not unfused).to_c()
        key = torch.zeros(2, dtype=torch.int64, device=dev)
        counts = torch.zeros(count, dtype=torch.int32, device=dev)
        plan.evaluate(pts, n, cfg, 0, count, key, counts)
        ref = oracle.f_counts(oracle.pack4(a, b), seed, 0, count, float(np.float32(thr * thr)),
                              oracle.f_kind(0, unfused))
        np.testing.assert_array_equal(counts.cpu().numpy(), ref)
        # (tiny: the 8-point sampler's absolute degeneracy tests reject every sample — parity only)
        assert case == "tiny" or (ref > 0).any()
    plan.close()


@pytest.mark.slow
def test_full_size_cfg4(torch_dev, oracle):
    """BASELINE config[3] at the bench's full size: F-RANSAC over 500k correspondences, 2^20 fixed
    hypotheses in one evaluate (bench.py's call at one rank). A 262144-hypothesis sample spread over
    the whole range (`_sample.bench_sample`: every 8-rank share's first and last 1024, 240 strided
    blocks, the bench's reported winner 1,028,871 and the device's argmax) equals the oracle count
    for count; the reduced key is the argmax of the device's own counts, the winner's mask holds
    exactly its count, and the host export sharded over 8 workspaces (deviceCount = 8; round-robin
    over the visible GPUs) is bit-identical to deviceCount = 1."""
    import _sample
    torch, dev = torch_dev
    from minicv_amd import device as D
    n, H = 500_000, 1 << 20
    a, b, _, _ = S.fundamental_problem(n, 4)
    thr = 5e-3
    pts = D.pack_points_tensor(a, b, dev)
    plan = D.RansacPlan(N.MODEL_FUNDAMENTAL, n, H)
    cfg = opencv.RansacParams(threshold=thr, seed=4, fixed_iters=True, max_iters=H).to_c()
    key = torch.zeros(2, dtype=torch.int64, device=dev)
    counts = torch.zeros(H, dtype=torch.int32, device=dev)
    plan.evaluate(pts, n, cfg, 0, H, key, counts)
    c = counts.cpu().numpy()
    cnt, idx = D.unpack_key(int(key[0].item()))
    assert cnt == c.max() and idx == int(np.argmax(c))
    assert idx == 1_028_871, "bench.py's reported cfg4 winner (profiles/r04_bench_fundamental.json)"
    p4 = oracle.pack4(a, b)
    thr2 = float(np.float32(thr * thr))
    ranges = _sample.bench_sample(H, around=(idx,))
    print("cfg4 sample:", _sample.describe(ranges))
    for lo, hi in ranges:   # OpenMP over the box's threads, ~5 s in all
        np.testing.assert_array_equal(c[lo:hi], oracle.f_counts(p4, 4, lo, hi - lo, thr2), err_msg=f"[{lo},{hi})")
    mask = torch.zeros(n, dtype=torch.uint8, device=dev)
    fc, F = plan.finalize(pts, n, opencv.RansacParams(threshold=thr, seed=4).to_c(), idx, mask)
    assert fc == cnt == int(mask.sum().item())
    plan.close()
    p1 = opencv.RansacParams(threshold=thr, seed=4, fixed_iters=True, max_iters=H)
    p8 = opencv.RansacParams(threshold=thr, seed=4, fixed_iters=True, max_iters=H, device_count=8)
    r1, r8 = opencv.findFundamentalMat(a, b, p1), opencv.findFundamentalMat(a, b, p8)
    assert r1[0] == r8[0] == cnt
    np.testing.assert_array_equal(r1[1], r8[1])
    np.testing.assert_array_equal(r1[2], r8[2])
    np.testing.assert_array_equal(r1[1], np.asarray(F).reshape(r1[1].shape))


# ---- OpenCV FM_RANSAC: 7-point minimal sets, up to 3 models per sample (MCV_FLAG_SEVEN_POINT) -----
@pytest.mark.parametrize("n,outl,seed,begin,count,error_kind,unfused", [
    (15, 0.0, 1, 0, 64, 1, True), (300, 0.5, 3, 0, 1024, 1, True), (2000, 0.5, 4, 77777, 512, 1, True),
    (1999, 0.5, 5, 0, 512, 0, True), (1000, 0.6, 6, 2**30, 256, 1, False), (64, 0.2, 8, 0, 300, 0, False)])
def test_f7_slot_counts_bit_exact(torch_dev, oracle, n, outl, seed, begin, count, error_kind, unfused):
    """Per-slot counts (3 model slots per hypothesis) equal the run7Point restatement's; the best key is
    the first maximum over slots."""
    torch, dev = torch_dev
    from minicv_amd import device as D
    a, b, _, _ = S.fundamental_problem(n, seed, outlier_frac=outl)
    pts = D.pack_points_tensor(a, b, dev)
    plan = D.RansacPlan(N.MODEL_FUNDAMENTAL, n, 3 * count)
    thr = 5e-3
    cfg = opencv.RansacParams(threshold=thr, seed=seed, error_kind=error_kind, fused_error=not unfused,
                              seven_point=True).to_c()
    key = torch.zeros(2, dtype=torch.int64, device=dev)
    counts = torch.zeros(3 * count, dtype=torch.int32, device=dev)
    plan.evaluate(pts, n, cfg, begin, count, key, counts)
    got = counts.cpu().numpy()
    ref = oracle.f7_counts(oracle.pack4(a, b), seed, begin, count, float(np.float32(thr * thr)),
                           oracle.f_kind(error_kind, unfused))
    np.testing.assert_array_equal(got, ref)
    if (ref >= 7).any() and not (ref == -2).any():
        c = ref.max()
        i = int(np.nonzero(ref == c)[0][0])
        assert int(key[0].item()) == (int(c) << 32) | (0xFFFFFFFF - (3 * begin + i))
    plan.close()


@pytest.mark.parametrize("n,outl,seed,iters,fixed", [(15, 0.0, 1, 200, False), (500, 0.5, 2, 1000, False),
                                                     (3000, 0.5, 3, 2000, False), (2000, 0.5, 4, 300, True)])
def test_find_fundamental7_vs_oracle(gpu, oracle, n, outl, seed, iters, fixed):
    """cvFindFundamentalMat with FM_RANSAC semantics (7-point sets, epipolar error, op-by-op): the
    winning slot, its F (no refit) and the mask equal the oracle's exactly."""
    a, b, inl, F = S.fundamental_problem(n, seed, outlier_frac=outl)
    p = opencv.RansacParams(threshold=5e-3, confidence=0.99, max_iters=iters, seed=seed, error_kind=N.FERR_EPIPOLAR,
                            seven_point=True, fixed_iters=fixed)
    cnt, Fg, mask = opencv.findFundamentalMat(a, b, p)
    rc, Fo, rmask, best = oracle.find_fundamental7(a, b, thr=5e-3, conf=0.99, max_iters=iters, seed=seed,
                                                   flags=N.FLAG_FIXED_ITERS if fixed else 0, error_kind=1)
    assert cnt == rc and best >= 0
    np.testing.assert_array_equal(Fg, Fo)
    np.testing.assert_array_equal(mask, rmask != 0)
    if n >= 500:   # the winning minimal-sample model (no refit, sigma 1e-3 vs thr 5e-3) keeps most
        assert mask[inl].mean() > 0.6 and mask[~inl].mean() < 0.05   # inliers (0.83 at seed 2)


def test_find_fundamental7_edges(gpu, oracle):
    a, b, _, F = S.fundamental_problem(7, 5, outlier_frac=0.0, sigma=0.0)
    p = opencv.RansacParams(threshold=5e-3, seven_point=True, error_kind=N.FERR_EPIPOLAR)
    cnt, Fg, mask = opencv.findFundamentalMat(a, b, p)      # N == 7: run7Point once, first model
    rc, Fo, rmask, _ = oracle.find_fundamental7(a, b, thr=5e-3)
    assert cnt == rc == 7 and mask.all()
    np.testing.assert_array_equal(Fg, Fo)
    a, b, _, _ = S.fundamental_problem(12, 5, outlier_frac=0.0)
    with pytest.raises(N.NativeError, match="N >= 15"):
        opencv.findFundamentalMat(a, b, p)


@pytest.mark.parametrize("seed", [41, 42, 43])
def test_f_eigen_minimal_solver_stress(torch_dev, oracle, seed):
    """run8Point's eigen-solve (JacobiImpl_ per lane) and its eigenvalue check against the oracle over
    many 8-point samples: every status and count identical."""
    torch, dev = torch_dev
    from minicv_amd import device as D
    rng = np.random.default_rng(seed)
    n = int(rng.integers(200, 2500))
    a, b, _, _ = S.fundamental_problem(n, seed, outlier_frac=float(rng.uniform(0.1, 0.7)))
    pts = D.pack_points_tensor(a, b, dev)
    count = 8192
    plan = D.RansacPlan(N.MODEL_FUNDAMENTAL, n, count)
    thr = 5e-3
    begin = int(rng.integers(0, 2**31))
    cfg = opencv.RansacParams(threshold=thr, seed=seed).to_c()
    key = torch.zeros(2, dtype=torch.int64, device=dev)
    counts = torch.zeros(count, dtype=torch.int32, device=dev)
    plan.evaluate(pts, n, cfg, begin, count, key, counts)
    got = counts.cpu().numpy()
    plan.close()
    ref = oracle.f_counts(oracle.pack4(a, b), seed, begin, count, float(np.float32(thr * thr)), oracle.f_kind(0, True))
    np.testing.assert_array_equal(got, ref)
