"""C-ABI boundary tests (CPU): libMiniCVNative.so loads, exports exactly what include/*.h declares
with the reference's names, marshals like the F# P/Invoke declarations (OpenCV.fs:339-382), and
its host-compiled twin of the per-hypothesis device code agrees with the oracle bit for bit.
No compute kernel is launched here."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

from minicv_amd import native as N
from minicv_amd import synthetic as S

ROOT = Path(__file__).resolve().parent.parent

REFERENCE_EXPORTS = ["cvRecoverPose", "cvRecoverPoses", "cvDetectFeatures", "cvFreeFeatures", "cvTest",
                     "cvFivePoint", "cvSolvePnP", "cvSolvePnPRansac", "cvRefinePnPLM", "cvRefinePnPVVS",
                     "solveAp3p", "cvDetectQRCode", "cvDetectArucoMarkers"]


def header_functions():
    names = []
    for h in (ROOT / "include").glob("*.h"):
        txt = h.read_text()
        names += re.findall(r"MCV_API\s+[\w\s\*]+?\b(\w+)\s*\(", txt)
    return sorted(set(names))


def test_header_declares_reference_surface():
    names = header_functions()
    for n in REFERENCE_EXPORTS:
        assert n in names, n
    for n in ("cvFindHomography", "cvFindFundamentalMat", "cvMatchHamming", "cvMatchL2"):
        assert n in names


def test_library_exports_every_declared_symbol(native):
    out = subprocess.run(["nm", "-D", "--defined-only", str(N.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [n for n in header_functions() if n not in exported]
    assert not missing, missing
    # unmangled C names, resolvable through ctypes like DllImport(EntryPoint=...)
    for n in header_functions():
        assert getattr(native.lib(), n) is not None
    # visibility=hidden: no C++ internals leak
    leaked = [s for s in exported if s.startswith("_ZN3mcv")]
    assert not leaked, leaked[:5]


def test_struct_layouts():
    assert C.sizeof(N.RecoverPoseConfig) == 40          # MiniCVNative.cpp:39-46
    assert C.sizeof(N.RansacConfig) == 48
    assert C.sizeof(N.M33d) == 72 and C.sizeof(N.V2d) == 16 and C.sizeof(N.V3d) == 24
    assert C.sizeof(N.ReplayState) == 24


def test_version_and_device_query(native):
    assert native.lib().mcvVersion().startswith(b"minicv-mi355x")
    assert native.lib().mcvDeviceCount() >= 0


def test_compute_fails_loudly_without_gpu(native):
    if native.lib().mcvDeviceCount() > 0:
        pytest.skip("a GPU is visible")
    src, dst, _ = S.homography_problem(50, 1)
    from minicv_amd import opencv
    with pytest.raises(N.NativeError, match="no HIP device"):
        opencv.findHomography(src, dst)
    with pytest.raises(N.NativeError, match="no HIP device"):
        opencv.matchHamming(np.zeros((4, 32), np.uint8), np.zeros((4, 32), np.uint8))


def test_out_of_scope_exports_fail_with_message(native):
    L = native.lib()
    assert L.cvDetectFeatures(None, 0, 0, 1, 1, None) is None
    assert "out" in native.last_error().lower() or "hot path" in native.last_error()
    cnt = C.c_int(7)
    assert not L.cvDetectQRCode(None, 0, 0, 1, None, C.addressof(cnt)) and cnt.value == 0
    L.cvTest()
    L.cvFreeFeatures(None)


def test_bad_arguments_rejected(native):
    L = native.lib()
    H = N.M33d()
    assert L.cvFindHomography(None, None, 10, None, C.addressof(H), None) == 0
    assert "null" in native.last_error()
    a = np.zeros((3, 2))
    m = np.zeros(3, np.uint8)
    assert L.cvFindHomography(a.ctypes.data, a.ctypes.data, 3, None, C.addressof(H), m.ctypes.data) == 0
    assert "at least 4" in native.last_error()


@pytest.mark.parametrize("ctr,key", [([0, 0, 0, 0], [0, 0]), ([1, 2, 3, 4], [5, 6]),
                                     ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2)])
def test_host_philox_matches_oracle(native, oracle, ctr, key):
    out = (C.c_uint32 * 4)()
    native.lib().mcvHostPhilox(*ctr, *key, out)
    assert list(out) == oracle.philox(ctr, key)


@pytest.mark.parametrize("fast", [False, True])
@pytest.mark.parametrize("n,outliers,seed", [(4, 0.0, 1), (7, 0.5, 2), (200, 0.5, 3), (5000, 0.7, 4)])
def test_host_hypothesis_bit_exact_vs_oracle(native, oracle, n, outliers, seed, fast):
    """The exact code the kernel runs (hyp_homography.h), compiled for the host, vs the independent
    C restatement: status, sample, fp64 model and fp32 model all bit-identical — for OpenCV's
    eigen-based runKernel (default) and the MCV_FLAG_FAST_MINIMAL elimination."""
    src, dst, _ = S.homography_problem(n, seed, outlier_frac=outliers)
    pts4 = oracle.pack4(src, dst)
    L = native.lib()
    H = np.zeros(9)
    hf = np.zeros(9, np.float32)
    idx = np.full(4, -1, np.int32)
    model = 0 | (0x100 if fast else 0)
    for hyp in list(range(300)) + [2**31 + 5, 2**32 - 1]:
        st = L.mcvHostHypothesis(model, pts4.ctypes.data, n, seed * 7919, hyp, H.ctypes.data, hf.ctypes.data,
                                 idx.ctypes.data)
        with oracle.fast_minimal(fast):
            st2, H2, hf2, idx2 = oracle.h_hypothesis(pts4, seed * 7919, hyp)
        assert st == st2
        if st == 1:
            np.testing.assert_array_equal(H, H2)
            np.testing.assert_array_equal(hf[:8], hf2)
            np.testing.assert_array_equal(idx, idx2)


def test_replay_chunks_match_oracle(native, oracle):
    rng = np.random.default_rng(3)
    L = native.lib()
    for trial in range(40):
        n = int(rng.integers(10, 1000))
        total = int(rng.integers(1, 3000))
        counts = rng.integers(-1, n + 1, size=total).astype(np.int32)
        if trial % 5 == 0:
            counts[rng.integers(0, total)] = -2
        fixed = bool(trial % 2)
        conf = float(rng.choice([0.9, 0.99, 0.995]))
        st = N.ReplayState()
        L.mcvReplayInit(C.addressof(st), total)
        begin = 0
        while begin < total and not st.stopped:
            c = int(rng.integers(1, 700))
            c = min(c, total - begin)
            chunk = np.ascontiguousarray(counts[begin:begin + c])
            L.mcvReplayChunk(C.addressof(st), chunk.ctypes.data, begin, c, n, 4, conf, int(fixed))
            begin += c
        best, bc = oracle.replay(counts, n, 4, conf, total, fixed)
        assert st.bestIndex == best
        if best >= 0:
            assert st.bestCount == bc


@pytest.mark.parametrize("fast", [False, True])
@pytest.mark.parametrize("n,outliers,seed", [(8, 0.0, 1), (9, 0.3, 2), (500, 0.5, 3), (5000, 0.7, 4)])
def test_host_f_hypothesis_bit_exact_vs_oracle(native, oracle, n, outliers, seed, fast):
    a, b, _, _ = S.fundamental_problem(n, seed, outlier_frac=outliers)
    pts4 = oracle.pack4(a, b)
    L = native.lib()
    F = np.zeros(9)
    Ff = np.zeros(9, np.float32)
    idx = np.full(8, -1, np.int32)
    model = 1 | (0x100 if fast else 0)
    for hyp in list(range(200)) + [2**32 - 7]:
        st = L.mcvHostHypothesis(model, pts4.ctypes.data, n, seed * 31, hyp, F.ctypes.data, Ff.ctypes.data,
                                 idx.ctypes.data)
        with oracle.fast_minimal(fast):
            st2, F2, idx2 = oracle.f_hypothesis(pts4, seed * 31, hyp)
        assert st == st2
        if st == 1:
            np.testing.assert_array_equal(F, F2)
            np.testing.assert_array_equal(idx, idx2)


def test_host_fingerprint_definition(native):
    """The plan guards' fingerprint (mcv_common.h fp_term: splitmix64 finalizer keyed by the word's
    position, summed mod 2^64) restated in Python; a rewrite, a swap of two words and a length change
    all change it."""
    import numpy as np
    M = (1 << 64) - 1

    def mix(z):
        z = (z + 0x9E3779B97F4A7C15) & M
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        return z ^ (z >> 31)

    rng = np.random.default_rng(1)
    w = rng.integers(0, 2**32, size=257, dtype=np.uint32)
    ref = sum(mix(mix(i) ^ int(x)) for i, x in enumerate(w)) & M
    fp = native.lib().mcvHostFingerprint
    assert fp(w.ctypes.data, w.nbytes) == ref
    w2 = w.copy()
    w2[[3, 4]] = w2[[4, 3]]
    assert fp(w2.ctypes.data, w2.nbytes) != ref
    assert fp(w.ctypes.data, w.nbytes - 4) != ref
    assert fp(w.ctypes.data, 0) == 0
