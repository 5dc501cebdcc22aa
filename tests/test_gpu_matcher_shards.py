"""GPU parity of the matchers at the shapes the multi-GPU runs launch (needs an MI355X).

`bench.py --gpus N` gives rank r the queries [shard(nq, r, N)) of BASELINE cfg2 (Hamming 10k x 10k)
and cfg5 (L2 50k x 50k x 128) against the whole replicated train set (bench.py:215-226); the
stream-K partitions of both GEMM forms (segment ranges, partial slots, the last-arrival folds) depend
on nq (csrc/match_l2.hip mcv_l2_gemm's partition, csrc/match_hamming.hip's), so every rank slice at
N = 2 / 4 / 8 is run here exactly as the bench runs it (device API, slice of the device tensor) and
checked against the oracle:
- Hamming: every query of every slice, all four outputs, bit for bit;
- L2: per N at least 1000 sampled queries spread over the slices plus each slice's first and last 64
  queries against oracle.match_l2, and every query of every slice against the full 50k call (the
  full call is itself sampled against the oracle in test_gpu_matchers.py).
The in-library multi-device exports (cvMatchHammingMulti / cvMatchL2Multi) must equal deviceCount 1
bit for bit; on a one-GPU box every block maps to device 0.
"""
import numpy as np
import pytest

from minicv_amd import dist as MD, native as N, opencv, synthetic as S

pytestmark = pytest.mark.gpu
RANKS = (2, 4, 8)


def _dev():
    import torch
    return torch.device("cuda:0")


def _run_slices(fn, qd, td, nq, world, dist_dtype):
    """Every rank's slice as bench.py runs it -> list of (begin, (idx, dist, idx2, dist2)) host arrays."""
    import torch
    dev = _dev()
    out = []
    for r in range(world):
        b0, cnt = MD.shard(nq, r, world)
        qs = qd[b0:b0 + cnt].contiguous()
        o = [torch.empty(cnt, dtype=torch.int32, device=dev), torch.empty(cnt, dtype=dist_dtype, device=dev),
             torch.empty(cnt, dtype=torch.int32, device=dev), torch.empty(cnt, dtype=dist_dtype, device=dev)]
        fn(qs, td, *o)
        torch.cuda.synchronize()
        out.append((b0, [x.cpu().numpy() for x in o]))
    return out


@pytest.fixture(scope="module")
def cfg2(oracle):
    q, t, _ = S.hamming_problem(10_000, 10_000, seed=2)
    return q, t, oracle.match_hamming(q, t)


@pytest.fixture(scope="module")
def cfg5():
    q, t, _ = S.l2_problem(50_000, 50_000, dim=128, seed=5)
    return q, t, opencv.matchL2(q, t)


@pytest.mark.parametrize("world", RANKS)
def test_hamming_rank_slices_cfg2(gpu, cfg2, world):
    """cfg2's 5000 / 2500 / 1250-query slices x 10k train: every query exact against the oracle."""
    import torch
    from minicv_amd import device as D
    q, t, ref = cfg2
    dev = _dev()
    qd, td = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
    for b0, got in _run_slices(D.match_hamming, qd, td, len(q), world, torch.int32):
        for g, r in zip(got, ref):
            np.testing.assert_array_equal(g, r[b0:b0 + len(g)])


def _l2_sample(nq, world, per_shape, edge, seed):
    """Indices: each slice's first / last `edge` queries + `per_shape` random ones over all slices."""
    pick = [np.random.default_rng(seed).choice(nq, size=per_shape, replace=False)]
    for r in range(world):
        b0, cnt = MD.shard(nq, r, world)
        pick += [np.arange(b0, b0 + min(edge, cnt)), np.arange(b0 + max(cnt - edge, 0), b0 + cnt)]
    return np.unique(np.concatenate(pick))


@pytest.mark.slow
@pytest.mark.parametrize("world", RANKS)
def test_l2_rank_slices_cfg5(gpu, oracle, cfg5, world):
    """cfg5's 25000 / 12500 / 6250-query slices x the full 50k train set: >= 1000 sampled queries per
    shape plus every slice's first and last 64 exactly against the oracle; every query of every slice
    equal to the single full-size call."""
    import torch
    from minicv_amd import device as D
    q, t, full = cfg5
    dev = _dev()
    qd, td = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
    slices = _run_slices(D.match_l2, qd, td, len(q), world, torch.float32)
    got = [np.concatenate([s[1][k] for s in slices]) for k in range(4)]
    assert sum(len(s[1][0]) for s in slices) == len(q)
    for g, f in zip(got, full):
        np.testing.assert_array_equal(g, f)
    pick = _l2_sample(len(q), world, 1000, 64, seed=world)
    ri, rd, ri2, rd2 = oracle.match_l2(q[pick], t)
    np.testing.assert_array_equal(got[0][pick], ri)
    np.testing.assert_array_equal(got[1][pick], rd.astype(np.float32))
    np.testing.assert_array_equal(got[2][pick], ri2)
    np.testing.assert_array_equal(got[3][pick], rd2.astype(np.float32))
    print(f"L2 world {world}: {len(pick)} sampled queries exact vs oracle; all {len(q)} equal to the full call")


@pytest.mark.parametrize("devices", [2, 3, 8])
def test_hamming_multi_device_equals_one(gpu, cfg2, devices):
    """cvMatchHammingMulti: query blocks over the devices (round-robin onto the visible ones), the
    result bit-identical to deviceCount 1 and to the oracle on cfg2."""
    q, t, ref = cfg2
    got = opencv.matchHamming(q, t, deviceCount=devices)
    one = opencv.matchHamming(q, t)
    for g, o, r in zip(got, one, ref):
        np.testing.assert_array_equal(g, o)
        np.testing.assert_array_equal(g, r)


@pytest.mark.parametrize("devices", [2, 3, 8])
def test_l2_multi_device_equals_one(gpu, oracle, devices):
    """cvMatchL2Multi on a cfg5 slice (the 8-rank share's 6250 queries x the full 50k train set):
    identical to deviceCount 1; 300 queries against the oracle."""
    q, t, _ = S.l2_problem(50_000, 50_000, dim=128, seed=5)
    q = q[:6250]
    got = opencv.matchL2(q, t, deviceCount=devices)
    one = opencv.matchL2(q, t)
    for g, o in zip(got, one):
        np.testing.assert_array_equal(g, o)
    pick = np.unique(np.r_[0:64, len(q) - 64:len(q), np.random.default_rng(devices).choice(len(q), 172, replace=False)])
    ri, rd, ri2, rd2 = oracle.match_l2(q[pick], t)
    np.testing.assert_array_equal(got[0][pick], ri)
    np.testing.assert_array_equal(got[2][pick], ri2)
    np.testing.assert_array_equal(got[1][pick], rd.astype(np.float32))


@pytest.mark.parametrize("nq,devices", [(1, 8), (5, 3), (17, 16)])
def test_multi_device_few_queries(gpu, oracle, nq, devices):
    """Fewer queries than devices: min(nq, deviceCount) blocks; both matchers still exact."""
    q, t, _ = S.hamming_problem(nq, 900, seed=nq)
    for g, r in zip(opencv.matchHamming(q, t, deviceCount=devices), oracle.match_hamming(q, t)):
        np.testing.assert_array_equal(g, r)
    lq, lt, _ = S.l2_problem(nq, 700, dim=128, seed=nq)
    ri, rd, ri2, rd2 = oracle.match_l2(lq, lt)
    i1, d1, i2, d2 = opencv.matchL2(lq, lt, deviceCount=devices)
    np.testing.assert_array_equal(i1, ri)
    np.testing.assert_array_equal(i2, ri2)
    np.testing.assert_array_equal(d1, rd.astype(np.float32))


def test_multi_device_rejects_bad_count(gpu):
    q, t, _ = S.hamming_problem(10, 10, seed=1)
    for bad in (0, 17):
        with pytest.raises(N.NativeError, match="deviceCount"):
            opencv.matchHamming(q, t, deviceCount=bad)


def test_matcher_stream_destroyed_between_calls(gpu, oracle):
    """a device-level match on a caller's stream that is destroyed right after the call,
    then a match on another stream: the library recorded its completion event when the first call
    left, so the second never touches the freed stream. Repeated for both matchers."""
    import gc
    import torch
    from minicv_amd import device as D
    dev = _dev()
    lq, lt, _ = S.l2_problem(1500, 3000, dim=128, seed=61)
    hq, ht, _ = S.hamming_problem(1500, 3000, seed=62)
    lqd, ltd = torch.from_numpy(lq).to(dev), torch.from_numpy(lt).to(dev)
    hqd, htd = torch.from_numpy(hq).to(dev), torch.from_numpy(ht).to(dev)
    li, lf = torch.empty(1500, dtype=torch.int32, device=dev), torch.empty(1500, dtype=torch.float32, device=dev)
    hi, hd = torch.empty(1500, dtype=torch.int32, device=dev), torch.empty(1500, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    for k in range(4):
        s = torch.cuda.Stream()
        D.match_l2(lqd, ltd, li, lf, stream=s)
        D.match_hamming(hqd, htd, hi, hd, stream=s)
        s.synchronize()
        del s                     # the caller's stream goes away (torch returns it to its pool)
        gc.collect()
        s2 = torch.cuda.Stream()
        D.match_l2(lqd, ltd, li, lf, stream=s2)
        D.match_hamming(hqd, htd, hi, hd, stream=s2)
        D.match_l2(lqd, ltd, li, lf)                   # and back to the default stream
        D.match_hamming(hqd, htd, hi, hd)
        torch.cuda.synchronize()
        del s2
    np.testing.assert_array_equal(li.cpu().numpy(), oracle.match_l2(lq, lt)[0])
    np.testing.assert_array_equal(hi.cpu().numpy(), oracle.match_hamming(hq, ht)[0])


def test_l2_raw_hip_stream_destroyed(gpu, oracle):
    """The same with a raw hipStream_t created and destroyed through the HIP runtime itself (torch
    pools its streams, so its `del` never frees the handle)."""
    import ctypes as C
    import torch
    from minicv_amd import device as D
    hip = C.CDLL("libamdhip64.so")
    dev = _dev()
    lq, lt, _ = S.l2_problem(800, 2000, dim=128, seed=63)
    lqd, ltd = torch.from_numpy(lq).to(dev), torch.from_numpy(lt).to(dev)
    li, lf = torch.empty(800, dtype=torch.int32, device=dev), torch.empty(800, dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    for k in range(3):
        h = C.c_void_p()
        assert hip.hipStreamCreateWithFlags(C.byref(h), 1) == 0
        ext = torch.cuda.ExternalStream(h.value)
        D.match_l2(lqd, ltd, li, lf, stream=ext)
        assert hip.hipStreamSynchronize(h) == 0
        assert hip.hipStreamDestroy(h) == 0
        D.match_l2(lqd, ltd, li, lf)       # next call on the default stream
        torch.cuda.synchronize()
    np.testing.assert_array_equal(li.cpu().numpy(), oracle.match_l2(lq, lt)[0])


def test_l2_single_train_row_has_no_second(gpu, oracle):
    """with nt = 1 the refine once folded the padding loads of its eight-partial
    batch as (+inf, real index) and returned idx2 = idx, dist2 = dist; the second place must stay
    empty: idx2 = -1, dist2 = +inf, as the oracle."""
    q, t, _ = S.l2_problem(300, 1, dim=128, seed=64)
    idx, d, idx2, d2 = opencv.matchL2(q, t)
    assert (idx == 0).all()
    assert (idx2 == -1).all() and np.isinf(d2).all()
    ri, rd, ri2, rd2 = oracle.match_l2(q, t)
    np.testing.assert_array_equal(idx2, ri2)
    np.testing.assert_array_equal(d2, rd2.astype(np.float32))


@pytest.mark.parametrize("nan_row", [0, 1])
def test_l2_two_train_rows_one_nan(gpu, oracle, nan_row):
    """nt = 2 with one NaN train row: one finite candidate only; the NaN row never enters the top-2
    (the oracle's strict <), so idx2 = -1 / dist2 = +inf."""
    q, t, _ = S.l2_problem(200, 2, dim=128, seed=65 + nan_row)
    t = t.copy()
    t[nan_row, 7] = np.nan
    idx, d, idx2, d2 = opencv.matchL2(q, t)
    ri, rd, ri2, rd2 = oracle.match_l2(q, t)
    np.testing.assert_array_equal(idx, ri)
    np.testing.assert_array_equal(idx2, ri2)
    np.testing.assert_array_equal(d, rd.astype(np.float32))
    np.testing.assert_array_equal(d2, rd2.astype(np.float32))
    assert (idx == 1 - nan_row).all()


@pytest.mark.slow
@pytest.mark.parametrize("devices", [2, 8])
def test_l2_multi_device_full_cfg5(gpu, cfg5, devices):
    """cvMatchL2Multi over BASELINE cfg5 at full size (50k x 50k): every output of every query equal to
    the single-device call (which test_l2_rank_slices_cfg5 / test_l2_full_size_cfg5 tie to the oracle)."""
    q, t, full = cfg5
    got = opencv.matchL2(q, t, deviceCount=devices)
    for g, f in zip(got, full):
        np.testing.assert_array_equal(g, f)
