"""The device API's stale-buffer guards (plan.h LastChunk, plan_guard.hip).

mcvRansacFinalize takes the winner's model from the last evaluated chunk's buffers when the winner lies
inside it; mcvRansacEvaluate / Finalize with MCV_FLAG_CV_SAMPLER reuse the plan's getSubset table for
hypotheses past 0. Both are keyed on the points' content (a device fingerprint), not only on the
pointer and N: a caller that rewrites the point buffer in place, or continues a search on another N,
gets the answer a fresh plan gives for the current points."""
import numpy as np
import pytest

from minicv_amd import native as N
from minicv_amd import opencv, synthetic as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev(gpu):
    import torch
    return torch, torch.device("cuda:0")


def _problem(model, n, seed, dev):
    """-> (device points, plan setup callback, threshold) of the model family."""
    from minicv_amd import device as D
    if model == N.MODEL_HOMOGRAPHY:
        src, dst, _ = S.homography_problem(n, seed)
        return D.pack_points_tensor(src, dst, dev), None, 5e-3
    if model == N.MODEL_FUNDAMENTAL:
        a, b, *_ = S.fundamental_problem(n, seed=seed)
        return D.pack_points_tensor(a, b, dev), None, 5e-3
    if model == N.MODEL_ESSENTIAL:
        a, b, *_ = S.essential_problem(n, seed=seed, outlier_frac=0.4)
        return D.pack_essential_tensor(a, b, 800.0, (640.0, 360.0), dev), None, 1.0 / 800.0
    img, W, _, K, d, *_ = S.pnp_problem(n, seed=seed, outlier_frac=0.4, dist=[-0.1, 0.02, 0.001, -0.001])
    return D.pack_pnp_tensor(img, W, dev), (K, d), 2.0


MODELS = [N.MODEL_HOMOGRAPHY, N.MODEL_FUNDAMENTAL, N.MODEL_ESSENTIAL, N.MODEL_PNP]


def _plan(model, n, hyps, cam):
    from minicv_amd import device as D
    p = D.RansacPlan(model, n, hyps)
    if cam is not None:
        p.set_camera(*cam)
    return p


def _finalize(plan, pts, n, cfg, idx, dev):
    import ctypes as C
    import torch
    mask = torch.zeros(n, dtype=torch.uint8, device=dev)
    m = (C.c_double * 9)()
    cnt = N.lib().mcvRansacFinalize(plan._p, pts.data_ptr(), n, C.addressof(cfg), int(idx), m, mask.data_ptr(),
                                    torch.cuda.current_stream().cuda_stream)
    N.check(cnt > 0, "mcvRansacFinalize")
    return cnt, np.array(m[:]), mask.cpu().numpy()


@pytest.mark.parametrize("model", MODELS)
def test_finalize_after_points_rewritten_in_place(torch_dev, model):
    """evaluate on points A, rewrite the same buffer with points B (same N), finalize the winner: the
    answer of a fresh plan on B (the winner re-solved from B), not the model cached from A."""
    torch, dev = torch_dev
    from minicv_amd import device as D
    n, hyps = 3000, 2048
    pts, cam, thr = _problem(model, n, 21, dev)
    ptsB, _, _ = _problem(model, n, 22, dev)
    slots = N.E_SLOTS if model == N.MODEL_ESSENTIAL else 1
    cfg = opencv.RansacParams(threshold=thr, seed=5, max_iters=hyps, fixed_iters=True).to_c()
    if model == N.MODEL_PNP:
        cfg.pnpKind = opencv.SOLVER_KIND["EPNP"]
    plan = _plan(model, n, hyps * slots, cam)
    key = torch.zeros(2, dtype=torch.int64, device=dev)
    plan.evaluate(pts, n, cfg, 0, hyps, key)
    cnt, idx = D.unpack_key(int(key.cpu()[0]))
    assert idx >= 0
    old = _finalize(plan, pts, n, cfg, idx, dev)          # cached path (points unchanged)
    plan.evaluate(pts, n, cfg, 0, hyps, key)
    pts.copy_(ptsB)                                       # in place: same pointer, same N
    fresh = _plan(model, n, hyps * slots, cam)
    try:
        ref = _finalize(fresh, pts, n, cfg, idx, dev)     # no chunk cached: the re-solve on B
    except N.NativeError:                                 # E: B's hypothesis has no model in that slot
        with pytest.raises(N.NativeError):
            _finalize(plan, pts, n, cfg, idx, dev)
        return
    got = _finalize(plan, pts, n, cfg, idx, dev)
    assert got[0] == ref[0]
    np.testing.assert_array_equal(got[1], ref[1])
    np.testing.assert_array_equal(got[2], ref[2])
    assert not np.array_equal(got[2], old[2]), "the rewrite should change the winner's mask"
    plan.close()
    fresh.close()


@pytest.mark.parametrize("model", MODELS)
def test_cv_table_continued_on_other_points(torch_dev, model):
    """a CV-sampler plan that evaluated [0, k) for N1 points, then [k, 2k) for a smaller N2
    (or, H / F, other points of the same N): the table is rebuilt, and the counts equal a fresh plan's
    [0, 2k) on the new points (no index >= N2 reaches the kernels)."""
    torch, dev = torch_dev
    slots = N.E_SLOTS if model == N.MODEL_ESSENTIAL else 1
    k = 512
    n1, n2 = 4000, 1500
    pts1, cam, thr = _problem(model, n1, 31, dev)
    cfg = opencv.RansacParams(threshold=thr, max_iters=2 * k, cv_sampler=True).to_c()
    if model == N.MODEL_PNP:
        cfg.pnpKind = opencv.SOLVER_KIND["EPNP"]
    cases = [(n2, 32)]
    if model in (N.MODEL_HOMOGRAPHY, N.MODEL_FUNDAMENTAL):
        cases.append((n1, 33))                        # same N, other points: checkSubset may differ
    for n_b, seed_b in cases:
        pts2, _, _ = _problem(model, n_b, seed_b, dev)
        plan = _plan(model, n1, 2 * k * slots, cam)
        key = torch.zeros(2, dtype=torch.int64, device=dev)
        c1 = torch.zeros(k * slots, dtype=torch.int32, device=dev)
        plan.evaluate(pts1, n1, cfg, 0, k, key, c1)
        c2 = torch.zeros(k * slots, dtype=torch.int32, device=dev)
        plan.evaluate(pts2, n_b, cfg, k, k, key, c2)
        fresh = _plan(model, n1, 2 * k * slots, cam)
        cr = torch.zeros(2 * k * slots, dtype=torch.int32, device=dev)
        fresh.evaluate(pts2, n_b, cfg, 0, 2 * k, key, cr)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(c2.cpu().numpy(), cr.cpu().numpy()[k * slots:])
        plan.close()
        fresh.close()


def test_device_fingerprint_equals_host(torch_dev):
    """The device kernel and the host twin compute the same fingerprint (a finalize after an unchanged
    evaluate takes the cached path only because they agree with themselves; this pins the definition)."""
    torch, dev = torch_dev
    import ctypes as C
    rng = np.random.default_rng(4)
    for nbytes in (4, 64, 4 * 1000, 16 * 100_003):
        a = rng.integers(0, 2**32, size=nbytes // 4, dtype=np.uint32)
        d = torch.from_numpy(a.view(np.int32)).to(dev)
        out = torch.zeros(1, dtype=torch.int64, device=dev)
        N.lib().mcvTestFingerprint(d.data_ptr(), nbytes, out.data_ptr())
        torch.cuda.synchronize()
        host = N.lib().mcvHostFingerprint(a.ctypes.data, nbytes)
        assert int(out.cpu()[0]) & 0xFFFFFFFFFFFFFFFF == host
