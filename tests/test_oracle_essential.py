"""Essential-matrix oracle (oracle/oracle_e.c) pinned on exact two-view geometry, and the product's
host-compiled twin (hyp_essential.h) against it bit for bit. CPU only.

Parity status: OpenCV is absent, so the five-point solver is pinned by ground truth:
for exact correspondences of a known pose the true E = [t]x R must be among the returned solutions,
and every solution must satisfy the essential-matrix constraints."""
import numpy as np
import pytest

from minicv_amd import synthetic as S
from minicv_amd import native as N

FOCAL, PP = 800.0, (640.0, 360.0)


def _skew(t):
    return np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])


def test_real_roots_known_polynomials(oracle):
    r = oracle.poly_real_roots(np.poly1d(np.arange(-4.5, 5.5, 1.0), r=True).coeffs[::-1])
    np.testing.assert_allclose(r, np.arange(-4.5, 5.5, 1.0), atol=1e-9)
    c = np.polymul(np.poly1d([1, -1, 0.5, 2], r=True).coeffs, [1, 0, 1])   # + complex pair +-i
    np.testing.assert_allclose(oracle.poly_real_roots(c[::-1]), [-1, 0.5, 1, 2], atol=1e-12)
    assert len(oracle.poly_real_roots(np.array([1.0, 0, 1.0]))) == 0       # z^2 + 1
    assert len(oracle.poly_real_roots(np.array([3.0]))) == 0
    np.testing.assert_allclose(oracle.poly_real_roots(np.array([-2.0, 1.0])), [2.0])
    # leading zeros trimmed
    np.testing.assert_allclose(oracle.poly_real_roots(np.array([-6.0, 1, 1, 0, 0])), [-3, 2], atol=1e-12)


def test_five_point_recovers_true_essential(oracle):
    """200 random exact poses: the true E is always among the solutions (the Nister formulation is
    ill-conditioned for a few configurations: all within 1e-4, >= 97% within 1e-8), and every
    solution satisfies the essential-matrix constraints."""
    devs = []
    for seed in range(200):
        rng = np.random.default_rng(1000 + seed)
        R = S.rotation(rng.normal(size=3), rng.uniform(0.02, 0.5))
        t = rng.normal(size=3)
        a, b, _, R, tu, E = S.essential_problem(5, seed=seed, outlier_frac=0, sigma=0, R=R, t=t + [0, 0, 0.3])
        p = oracle.pack_e(a, b, FOCAL, PP)
        Es = oracle.e_solve5(p[:, 0], p[:, 1], p[:, 2], p[:, 3])
        assert 1 <= len(Es) <= 10
        devs.append(min(min(np.abs(e - E).max(), np.abs(e + E).max()) for e in Es))
        x1 = np.c_[p[:, :2], np.ones(5)]
        x2 = np.c_[p[:, 2:], np.ones(5)]
        for e in Es:
            assert abs(np.linalg.norm(e) - 1) < 1e-12
            assert abs(np.linalg.det(e)) < 1e-6
            np.testing.assert_allclose(2 * e @ e.T @ e - np.trace(e @ e.T) * e, 0, atol=1e-5)
            np.testing.assert_allclose(np.einsum("ij,jk,ik->i", x2, e, x1), 0, atol=1e-6)
    devs = np.array(devs)
    assert devs.max() < 1e-4 and np.mean(devs < 1e-8) >= 0.97 and np.median(devs) < 1e-12


def test_decompose_gives_true_pose(oracle):
    _, _, _, R, tu, E = S.essential_problem(5, seed=3, outlier_frac=0)
    for sgn in (1, -1):
        R1, R2, t = oracle.e_decompose(sgn * E)
        for Rk in (R1, R2):
            np.testing.assert_allclose(Rk @ Rk.T, np.eye(3), atol=1e-12)
            assert abs(np.linalg.det(Rk) - 1) < 1e-12
        assert min(np.abs(R1 - R).max(), np.abs(R2 - R).max()) < 1e-12
        assert min(np.abs(t - tu).max(), np.abs(t + tu).max()) < 1e-12
        # E ~ [t]x R1 up to sign
        Ep = _skew(t) @ R1
        Ep /= np.linalg.norm(Ep)
        assert min(np.abs(Ep - sgn * E).max(), np.abs(Ep + sgn * E).max()) < 1e-12


def test_find_essential_and_recover_pose_synthetic(oracle):
    a, b, inl, R, tu, E = S.essential_problem(2000, seed=11, outlier_frac=0.4, sigma=0.2)
    cnt, Ee, mask, best = oracle.find_essential(a, b, FOCAL, PP, thr=1.0, conf=0.999, max_iters=1000, seed=5)
    assert cnt == mask.sum() and cnt > 0.85 * inl.sum()
    assert ((mask != 0) & ~inl).sum() < 0.01 * len(a)
    assert min(np.abs(Ee - E).max(), np.abs(Ee + E).max()) < 0.05
    res, Rr, tr, g = oracle.recover_pose(a, b, Ee, mask, FOCAL, PP)
    assert res == g.max() and res > 0.95 * cnt
    assert np.abs(Rr - R).max() < 0.02 and np.abs(tr - tu).max() < 0.05


def test_replay_slots_semantics(oracle):
    # models of one hypothesis are tried in order; the first strictly better wins
    c = np.full(3 * 10, -1, np.int32)
    c[0:3] = [7, 9, 9]
    c[10:12] = [9, 12]
    c[20] = 12
    best, bc = oracle.replay_slots(c, 3, 100, 5, 0.99, 3, True)
    assert best == 11 and bc == 12
    c[20] = -2                                           # sampler failure stops the loop
    c[10:12] = [3, 4]
    best, bc = oracle.replay_slots(c, 3, 100, 5, 0.99, 3, True)
    assert best == 1 and bc == 9


# ---- product host twin (hyp_essential.h compiled for x86) vs the oracle ------------------------
def test_host_five_point_bit_exact(native, oracle):
    rng = np.random.default_rng(7)
    L = native.lib()
    for trial in range(150):
        if trial % 3 == 0:
            p = rng.normal(size=(5, 4))                           # arbitrary (noisy) coordinates
        else:
            a, b, *_ = S.essential_problem(5, seed=trial, outlier_frac=0, sigma=0.5)
            p = oracle.pack_e(a, b, FOCAL, PP)
        p20 = np.ascontiguousarray(np.concatenate([p[:, 0], p[:, 1], p[:, 2], p[:, 3]]))
        E90 = np.zeros(90)
        n = L.mcvHostFivePoint(p20.ctypes.data, E90.ctypes.data)
        Es = oracle.e_solve5(p[:, 0], p[:, 1], p[:, 2], p[:, 3])
        assert n == len(Es)
        np.testing.assert_array_equal(E90.reshape(10, 3, 3)[:n], Es)


@pytest.mark.parametrize("n,outliers,seed", [(5, 0.0, 1), (6, 0.3, 2), (300, 0.5, 3), (5000, 0.6, 4)])
def test_host_essential_hypothesis_bit_exact(native, oracle, n, outliers, seed):
    a, b, *_ = S.essential_problem(n, seed=seed, outlier_frac=outliers)
    p = oracle.pack_e(a, b, FOCAL, PP)
    L = native.lib()
    for hyp in list(range(150)) + [2**32 - 3]:
        E2, idx2 = np.zeros(90), np.zeros(5, np.int32)
        n2 = L.mcvHostEssential(p.ctypes.data, n, seed * 3, hyp, E2.ctypes.data, idx2.ctypes.data)
        n1, E1, idx1 = oracle.e_hypothesis(p, seed * 3, hyp)
        assert n1 == n2
        np.testing.assert_array_equal(E1.ravel(), E2)
        if n1 >= 0:
            np.testing.assert_array_equal(idx1, idx2)


def test_host_decompose_bit_exact(native, oracle):
    L = native.lib()
    for s in range(20):
        _, _, _, _, _, E = S.essential_problem(5, seed=s)
        E = np.ascontiguousarray((E + np.random.default_rng(s).normal(0, 1e-3, (3, 3))).ravel())
        r1, r2, t = np.zeros(9), np.zeros(9), np.zeros(3)
        L.mcvHostDecomposeEssential(E.ctypes.data, r1.ctypes.data, r2.ctypes.data, t.ctypes.data)
        R1, R2, t0 = oracle.e_decompose(E)
        np.testing.assert_array_equal(r1, R1.ravel())
        np.testing.assert_array_equal(r2, R2.ravel())
        np.testing.assert_array_equal(t, t0)


def test_replay_models_export_matches_oracle(native, oracle):
    import ctypes as C
    rng = np.random.default_rng(9)
    L = native.lib()
    for trial in range(30):
        n = int(rng.integers(10, 500))
        nh = int(rng.integers(1, 800))
        c = np.full(nh * 10, -1, np.int32)
        k = rng.integers(0, 5, size=nh)
        for h in range(nh):
            c[10 * h:10 * h + k[h]] = rng.integers(0, n + 1, size=k[h])
        if trial % 4 == 0:
            c[10 * int(rng.integers(0, nh))] = -2
        fixed = bool(trial % 2)
        st = N.ReplayState()
        L.mcvReplayInit(C.addressof(st), nh)
        begin = 0
        while begin < nh and not st.stopped:
            cnt = min(int(rng.integers(1, 200)), nh - begin)
            chunk = np.ascontiguousarray(c[10 * begin:10 * (begin + cnt)])
            L.mcvReplayChunkModels(C.addressof(st), chunk.ctypes.data, begin, cnt, 10, n, 5, 0.99, int(fixed))
            begin += cnt
        best, bc = oracle.replay_slots(c, nh, n, 5, 0.99, nh, fixed)
        assert st.bestIndex == best
        if best >= 0:
            assert st.bestCount == bc


def _host_roots(native, c, fixed):
    import ctypes as C
    c = np.ascontiguousarray(c, dtype=np.float64)
    r = np.zeros(10, dtype=np.float64)
    n = native.lib().mcvHostRealRoots(c.ctypes.data_as(C.c_void_p), len(c) - 1, int(fixed),
                                      r.ctypes.data_as(C.c_void_p))
    assert n >= 0
    return r[:n]


def test_host_real_roots_fixed_form_bit_exact(native, oracle):
    """The register-resident fixed-size root finder (AP3P's quartic) equals the generic one and the
    oracle bit for bit: random quartics, leading zeros (degree 3..0), repeated and clustered roots,
    zero / huge / tiny coefficients, non-finite input."""
    rng = np.random.default_rng(7)
    cases = [rng.normal(size=5) * 10.0 ** rng.integers(-6, 7, size=5) for _ in range(3000)]
    cases += [np.poly1d(rng.normal(size=4), r=True).coeffs[::-1] for _ in range(500)]
    cases += [np.poly1d([r, r, s, s], r=True).coeffs[::-1] for r, s in rng.normal(size=(300, 2))]
    cases += [np.poly1d([1.0, 1.0 + 1e-12, -2.0, 3.0], r=True).coeffs[::-1]]
    for d in range(4):
        cases += [np.concatenate([rng.normal(size=d + 1), np.zeros(4 - d)]) for _ in range(100)]
    cases += [np.array([0.0, 0, 0, 0, 0]), np.array([1.0, 0, 0, 0, 1e-300]), np.array([1e300, -1e300, 1, 0, 1]),
              np.array([np.nan, 1, 2, 3, 4]), np.array([1, 2, 3, 4, np.inf]), np.array([-1.0, 0, 0, 0, 1])]
    for c in cases:
        c = np.asarray(c, dtype=np.float64)
        fx = _host_roots(native, c, True)
        gen = _host_roots(native, c, False)
        np.testing.assert_array_equal(fx, gen)
        np.testing.assert_array_equal(fx, oracle.poly_real_roots(c))


# ---- cvFivePoint's own path (fivepoint.cpp:233-339; oracle orc_e_solve5_ref) ---------------------
def test_solve_poly_durand_kerner(oracle):
    """cv::solvePoly restated (Durand-Kerner, 300 sweeps): the root set of random degree-10
    polynomials equals numpy's companion-matrix roots; real roots come out with |Im| ~ 0."""
    rng = np.random.default_rng(3)
    for _ in range(100):
        real = np.sort(rng.uniform(-3, 3, size=rng.integers(0, 6) * 2))
        cplx = rng.normal(size=(5 - len(real) // 2)) + 1j * rng.uniform(0.2, 2, size=5 - len(real) // 2)
        rts = np.concatenate([real, cplx, cplx.conj()])
        c = np.real(np.poly(rts))[::-1] * rng.uniform(0.5, 2)          # ascending coefficients
        got = oracle.solve_poly10(c)
        for r in rts:
            assert np.min(np.abs(got - r)) < 1e-7 * max(1, abs(r))
        assert (np.abs(got.imag[np.abs(got.imag) < 1e-6]) <= 1e-10).all()


def test_five_point_ref_recovers_true_essential(oracle):
    """The export path finds the true E for exact poses and agrees with the RANSAC solver's model set
    (same count, same E up to sign: median ~1e-14, 95% within 1e-9, all within 1e-4 — the Nister
    formulation is ill-conditioned for a few configurations); every solution has unit norm."""
    worst, extra, devs = 0.0, 0, []
    for seed in range(200):
        rng = np.random.default_rng(1000 + seed)
        R = S.rotation(rng.normal(size=3), rng.uniform(0.02, 0.5))
        t = rng.normal(size=3)
        a, b, _, R, tu, E = S.essential_problem(5, seed=seed, outlier_frac=0, sigma=0, R=R, t=t + [0, 0, 0.3])
        p = oracle.pack_e(a, b, FOCAL, PP)
        Er = oracle.e_solve5_ref(p[:, 0], p[:, 1], p[:, 2], p[:, 3])
        Es = oracle.e_solve5(p[:, 0], p[:, 1], p[:, 2], p[:, 3])
        assert 1 <= len(Er) <= 10
        worst = max(worst, min(min(np.abs(e - E).max(), np.abs(e + E).max()) for e in Er))
        for e in Er:
            np.testing.assert_allclose(np.linalg.norm(e), 1.0, atol=1e-12)
        assert len(Er) == len(Es)
        for e in Es:   # every RANSAC-path model is among the export's (up to sign)
            devs.append(min(min(np.abs(e - f).max(), np.abs(e + f).max()) for f in Er))
    assert worst < 1e-4 and max(devs) < 1e-4 and np.quantile(devs, 0.95) < 1e-9


def test_host_five_point_ref_bit_exact(native, oracle):
    rng = np.random.default_rng(8)
    L = native.lib()
    for trial in range(150):
        if trial % 3 == 0:
            p = rng.normal(size=(5, 4))
        else:
            a, b, *_ = S.essential_problem(5, seed=trial, outlier_frac=0, sigma=0.5)
            p = oracle.pack_e(a, b, FOCAL, PP)
        p20 = np.ascontiguousarray(np.concatenate([p[:, 0], p[:, 1], p[:, 2], p[:, 3]]))
        E90 = np.zeros(90)
        n = L.mcvHostFivePointRef(p20.ctypes.data, E90.ctypes.data)
        Es = oracle.e_solve5_ref(p[:, 0], p[:, 1], p[:, 2], p[:, 3])
        assert n == len(Es)
        np.testing.assert_array_equal(E90.reshape(10, 3, 3)[:n], Es)
