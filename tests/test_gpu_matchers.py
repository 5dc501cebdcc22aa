"""GPU parity of the brute-force matchers against the oracle (needs an MI355X).
Hamming: integer work, bit-exact (indices, distances, second best, lowest-index tie-break).
"""
from pathlib import Path

import numpy as np
import pytest

from minicv_amd import native as N, opencv, synthetic as S

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


# ---- L2 (fp32 MFMA GEMM form, exact re-rank) ------------------------------------------------
# Exact bar: the GEMM form only nominates candidates; mcv_l2_refine / mcv_l2_exact_scan decide with
# the oracle's exact definition (fp64 differences, sequential sum, ties -> lowest index), so idx /
# idx2 equal the oracle's and dist / dist2 are (float)sqrt of the same fp64 sums, bit for bit.


def check_l2(oracle, q, t):
    idx, d, idx2, d2 = opencv.matchL2(q, t)
    ri, rd, ri2, rd2 = oracle.match_l2(q, t)
    np.testing.assert_array_equal(idx, ri)
    np.testing.assert_array_equal(d, rd.astype(np.float32))
    # every shape, nt = 1 included (the second place must stay -1 / +inf there)
    np.testing.assert_array_equal(idx2, ri2)
    np.testing.assert_array_equal(d2, rd2.astype(np.float32))
    return 1.0


def test_l2_golden(gpu, oracle):
    g = np.load(GOLDEN / "matchers.npz")
    idx, d, idx2, d2 = opencv.matchL2(g["lq"], g["lt"])
    np.testing.assert_array_equal(idx, g["l_idx"])
    np.testing.assert_array_equal(idx2, g["l_idx2"])
    np.testing.assert_array_equal(d, g["l_dist"].astype(np.float32))
    np.testing.assert_array_equal(d2, g["l_dist2"].astype(np.float32))


def test_l2_near_ties_take_the_exact_scan(gpu, oracle):
    """Train sets built of near-duplicates (perturbations below the GEMM form's rounding) force the
    exact scan; the answer still equals the oracle's exactly."""
    rng = np.random.default_rng(11)
    base = S.sift_like(300, 128, rng)
    t = np.concatenate([base, base + rng.normal(scale=1e-4, size=base.shape).astype(np.float32),
                        base + np.float32(1e-3)]).astype(np.float32)
    q = (base[rng.integers(0, 300, size=500)] + rng.normal(scale=0.5, size=(500, 128))).astype(np.float32)
    check_l2(oracle, q, t)


@pytest.mark.parametrize("offset", [0.0, 1000.0])
def test_l2_exact_scan_filter_near_threshold(gpu, oracle, offset):
    """The exact scan's fp32 filter against rows whose distances sit within fp32 rounding of the
    filter bound: clusters of near-duplicates (perturbations of 1e-3 on values up to 1000 + 255) around
    each query's true neighbours; every decision still equals the oracle's exact answer."""
    rng = np.random.default_rng(29)
    base = S.sift_like(200, 128, rng).astype(np.float64) + offset
    t = np.concatenate([base + rng.normal(scale=1e-3, size=base.shape) for _ in range(6)]).astype(np.float32)
    q = (base[rng.integers(0, 200, size=700)] + rng.normal(scale=2e-3, size=(700, 128))).astype(np.float32)
    check_l2(oracle, q, t)
    assert N.lib().mcvL2LastExactScans() > 0


@pytest.mark.parametrize("nq,nt,dim", [(1, 1, 128), (1, 2, 128), (33, 31, 128), (200, 777, 128), (129, 4099, 128),
                                       (300, 500, 64), (100, 300, 32), (100, 300, 17), (64, 200, 256),
                                       (250, 333, 61)])
def test_l2_shapes(gpu, oracle, nq, nt, dim):
    q, t, _ = S.l2_problem(nq, nt, dim=dim, seed=nq + nt + dim)
    check_l2(oracle, q, t)


def test_l2_duplicated_train_exact_scan_cost(gpu, oracle):
    """Repeated-texture train sets: every query's best and second best are exact duplicates, so the GEMM
    form cannot separate them and every query takes the exact scan (O(nq nt dim) fp64). The answer is still
    the oracle's, and the queue length and the call's time are reported (the ADVICE r02 worst case)."""
    import time
    rng = np.random.default_rng(17)
    base = S.sift_like(500, 128, rng)
    t = np.concatenate([base] * 8).astype(np.float32)                       # 4000 rows, 500 distinct
    q = (base[rng.integers(0, 500, size=2000)] + rng.normal(scale=0.3, size=(2000, 128))).astype(np.float32)
    opencv.matchL2(q, t)                                                    # warm-up
    t0 = time.perf_counter()
    check_l2(oracle, q, t)
    scans = N.lib().mcvL2LastExactScans()
    print(f"duplicated train: {scans} of {len(q)} queries took the exact scan; "
          f"match + oracle check {time.perf_counter() - t0:.3f} s")
    assert scans >= 0.9 * len(q)


@pytest.mark.parametrize("scale,shift", [(1.0, 0.0), (32767.0 / 255.0, 0.0), (32768.0 / 255.0, 0.0), (1e4, 0.0),
                                         (1e-6, 0.0), (3e-9, 0.0), (1.0, -127.5), (2.0 ** -20, 2.0 ** -20)])
def test_l2_f16_split_domain(gpu, oracle, scale, shift):
    """The f16-split GEMM form runs while every |x| < 2^15 (the first two scales, the tiny ones whose
    split parts are f16 subnormals, signed data); at max |x| = 2^15 and above the f32 form takes the
    launch (device-side flag). Either way the answer is the oracle's, bit for bit."""
    q, t, _ = S.l2_problem(300, 1200, dim=128, seed=23)
    q = (q.astype(np.float64) * scale + shift).astype(np.float32)
    t = (t.astype(np.float64) * scale + shift).astype(np.float32)
    if scale == 32768.0 / 255.0:
        t[0, 0] = np.float32(32768.0)   # exactly at the bound: out of the f16 domain
    check_l2(oracle, q, t)


@pytest.mark.parametrize("dim", [128, 200])
def test_l2_non_finite_coordinates(gpu, oracle, dim):
    """NaN / inf coordinates in some queries and train rows (the f32 GEMM form takes the launch): a NaN
    distance never enters a top-2 (the oracle's strict < in index order), +inf distances rank last."""
    q, t, _ = S.l2_problem(300, 900, dim=dim, seed=31)
    q, t = q.copy(), t.copy()
    q[5, 3] = np.nan
    q[7, :] = np.nan
    t[11, 0] = np.nan
    t[13, 2] = np.inf
    t[17, :] = np.inf
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
    check_l2(oracle, q, t)
    idx = opencv.matchL2(q, t)[0]
    ok = planted >= 0
    assert np.mean(idx[ok] == planted[ok]) > 0.99


@pytest.mark.slow
def test_l2_full_size_cfg5(gpu, oracle):
    """BASELINE config[4] at full size (50k x 50k SIFT-128 fp32): 4000 sampled queries plus the first
    and last 64 exactly equal to the oracle (indices and distances bit for bit), planted-neighbour
    recall, determinism. The multi-GPU rank slices: test_gpu_matcher_shards.py."""
    q, t, planted = S.l2_problem(50_000, 50_000, dim=128, seed=5)
    idx, d, idx2, d2 = opencv.matchL2(q, t)
    rng = np.random.default_rng(0)
    pick = np.unique(np.r_[0:64, 50_000 - 64:50_000, rng.choice(50_000, size=4000, replace=False)])
    ri, rd, ri2, rd2 = oracle.match_l2(q[pick], t)
    np.testing.assert_array_equal(idx[pick], ri)
    np.testing.assert_array_equal(idx2[pick], ri2)
    np.testing.assert_array_equal(d[pick], rd.astype(np.float32))
    np.testing.assert_array_equal(d2[pick], rd2.astype(np.float32))
    ok = planted >= 0
    assert np.mean(idx[ok] == planted[ok]) > 0.99
    again = opencv.matchL2(q, t)
    np.testing.assert_array_equal(again[0], idx)
    np.testing.assert_array_equal(again[1], d)


@pytest.mark.parametrize("nt", [1, 2, 3])
def test_l2_fp32_norm_overflow_few_train(gpu, oracle, nt):
    """coordinates around 1e20 overflow the fp32 norms (every GEMM score inf) while the fp64
    distances stay finite; with nt <= 2 the refine step once certified the empty candidate list. A query
    without both candidates now takes the exact scan: the oracle's finite answer."""
    rng = np.random.default_rng(40 + nt)
    q = (rng.normal(size=(70, 128)) * 1e20).astype(np.float32)
    t = (rng.normal(size=(nt, 128)) * 1e20).astype(np.float32)
    check_l2(oracle, q, t)
    idx = opencv.matchL2(q, t)[0]
    assert (idx >= 0).all()


def test_matchers_back_to_back_on_two_streams(gpu, oracle):
    """the device-level matchers are asynchronous on the caller's stream and share one
    workspace per thread and device; two calls on different streams, issued back to back without a
    synchronisation, must not race (StreamFence orders them)."""
    import torch
    from minicv_amd import device as D
    dev = torch.device("cuda:0")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    qa, ta, _ = S.l2_problem(3000, 5000, dim=128, seed=51)
    qb, tb, _ = S.l2_problem(2000, 7000, dim=128, seed=52)
    ha, hta, _ = S.hamming_problem(3000, 4000, seed=53)
    hb, htb, _ = S.hamming_problem(2500, 6000, seed=54)
    out = {}
    for name, (q, t, fn, dt) in {"l2a": (qa, ta, D.match_l2, torch.float32), "l2b": (qb, tb, D.match_l2, torch.float32),
                                 "ha": (ha, hta, D.match_hamming, torch.int32),
                                 "hb": (hb, htb, D.match_hamming, torch.int32)}.items():
        qd, td = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
        out[name] = (qd, td, fn, torch.empty(len(q), dtype=torch.int32, device=dev),
                     torch.empty(len(q), dtype=dt, device=dev))
    torch.cuda.synchronize()
    for k in range(3):
        for name, s in (("l2a", s1), ("l2b", s2), ("ha", s1), ("hb", s2)):
            qd, td, fn, idx, dist = out[name]
            with torch.cuda.stream(s):
                fn(qd, td, idx, dist, stream=s)
    torch.cuda.synchronize()
    for name, (q, t) in {"l2a": (qa, ta), "l2b": (qb, tb)}.items():
        ri, rd, _, _ = oracle.match_l2(q[:300], t)
        np.testing.assert_array_equal(out[name][3].cpu().numpy()[:300], ri)
    for name, (q, t) in {"ha": (ha, hta), "hb": (hb, htb)}.items():
        ri, rd, _, _ = oracle.match_hamming(q, t)
        np.testing.assert_array_equal(out[name][3].cpu().numpy(), ri)


@pytest.fixture(params=["gemm", "popcount"])
def hamming_form(request):
    """Both Hamming kernel forms: the fp4 GEMM on the matrix cores (the default of every entry point)
    and the XOR / popcount sweep, chosen through mcvMatchHammingDeviceForm."""
    return request.param


def check_hamming_form(oracle, form, q, t):
    """The device entry point with an explicit kernel form against the oracle (all four outputs)."""
    import torch
    from minicv_amd import device as D
    dev = torch.device("cuda:0")
    nq = q.shape[0]
    tq, tt = torch.from_numpy(np.ascontiguousarray(q)).to(dev), torch.from_numpy(np.ascontiguousarray(t)).to(dev)
    idx, dist, idx2, dist2 = (torch.empty(nq, dtype=torch.int32, device=dev) for _ in range(4))
    D.match_hamming(tq, tt, idx, dist, idx2, dist2, form=form)
    torch.cuda.synchronize()
    for g, r in zip((idx, dist, idx2, dist2), oracle.match_hamming(q, t)):
        np.testing.assert_array_equal(g.cpu().numpy(), r)
    return idx.cpu().numpy(), dist.cpu().numpy(), idx2.cpu().numpy(), dist2.cpu().numpy()


@pytest.mark.parametrize("nq,nt,nbytes", [(1, 1, 32), (33, 31, 32), (257, 1000, 16), (300, 333, 61), (513, 4099, 64),
                                          (1000, 70000, 32)])
def test_hamming_forms_agree(gpu, oracle, hamming_form, nq, nt, nbytes):
    q, t, _ = S.hamming_problem(nq, nt, nbytes=nbytes, seed=3 * nq + nt)
    check_hamming_form(oracle, hamming_form, q, t)


@pytest.mark.parametrize("nbytes", [32, 64])
def test_hamming_extreme_distances(gpu, oracle, hamming_form, nbytes):
    """All-zero / all-one descriptors: distances 0 and the maximum 8 * nbytes (the GEMM form's accumulator
    at 2 Kp, its key at 2^31 + index), ties at the maximum broken by the lowest index."""
    rng = np.random.default_rng(nbytes)
    t = rng.integers(0, 256, size=(3000, nbytes), dtype=np.uint8)
    t[:100] = 0
    t[100:200] = 255
    q = np.concatenate([np.zeros((40, nbytes), np.uint8), np.full((40, nbytes), 255, np.uint8),
                        rng.integers(0, 256, size=(50, nbytes), dtype=np.uint8)])
    t2 = np.full((5, nbytes), 255, np.uint8)          # every query at one distance from all of them
    check_hamming_form(oracle, hamming_form, q, t)
    idx, dist, idx2, dist2 = check_hamming_form(oracle, hamming_form, q[:40], t2)
    assert (dist == 8 * nbytes).all() and (idx == 0).all() and (idx2 == 1).all()


def test_hamming_gemm_long_ranges(gpu, oracle):
    """A call large enough that the GEMM form's stream-K ranges reach their 128-tile cap (the key's
    4096-row index field) and the grid exceeds the resident slots: 8000 x 120000 (32 query blocks x
    3750 tiles -> 938 ranges of <= 128 tiles). Every query against the popcount form (an independent
    kernel) and a sample of 400 queries against the oracle."""
    import torch
    from minicv_amd import device as D
    q, t, _ = S.hamming_problem(8000, 120_000, seed=11)
    dev = torch.device("cuda:0")
    tq, tt = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
    outs = {}
    for form in ("gemm", "popcount"):
        o = [torch.empty(q.shape[0], dtype=torch.int32, device=dev) for _ in range(4)]
        D.match_hamming(tq, tt, *o, form=form)
        torch.cuda.synchronize()
        outs[form] = [x.cpu().numpy() for x in o]
    for g, p in zip(outs["gemm"], outs["popcount"]):
        np.testing.assert_array_equal(g, p)
    sel = np.random.default_rng(0).choice(q.shape[0], 400, replace=False)
    for g, r in zip(outs["gemm"], oracle.match_hamming(q[sel], t)):
        np.testing.assert_array_equal(g[sel], r)
