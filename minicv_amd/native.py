"""ctypes binding of libMiniCVNative.so — the same entry points the F# `module OpenCV.Native`
binds with [<DllImport("MiniCVNative")>] (/root/reference/src/MiniCV/OpenCV.fs:339-382), plus the
new hot-path exports declared in include/minicv_native.h.

The library is the product: there is no Python or CPU fallback. If it is missing, importing the
binding raises. Build it with `python -m minicv_amd.build` (or __graft_entry__.build()).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
LIB_PATH = Path(os.environ.get("MINICV_NATIVE_LIB",
                               ROOT / "libs" / "Native" / "MiniCV" / "linux" / "AMD64" / "libMiniCVNative.so"))


class V2d(C.Structure):
    _fields_ = [("X", C.c_double), ("Y", C.c_double)]


class V3d(C.Structure):
    _fields_ = [("X", C.c_double), ("Y", C.c_double), ("Z", C.c_double)]


class M33d(C.Structure):
    _fields_ = [("M", C.c_double * 9)]


class Camera(C.Structure):
    """mcvCamera: the MiniCV Camera record (src/MiniCV/Camera.fs:7-14), field order kept."""
    _fields_ = [("location", V3d), ("forward", V3d), ("up", V3d), ("right", V3d), ("focal", V2d)]


class RecoverPoseConfig(C.Structure):
    """MiniCVNative.cpp:39-46 / OpenCV.fs:16-36."""
    _fields_ = [("FocalLength", C.c_double), ("PrincipalPoint", V2d), ("Probability", C.c_double),
                ("InlierThreshold", C.c_double)]


class RansacConfig(C.Structure):
    _fields_ = [("threshold", C.c_double), ("confidence", C.c_double), ("maxIters", C.c_int),
                ("method", C.c_int), ("seed", C.c_uint64), ("deviceCount", C.c_int), ("flags", C.c_int),
                ("errorKind", C.c_int), ("pnpKind", C.c_int)]


class KeyPoint2d(C.Structure):
    """MiniCVNative.h:14-21 / OpenCV.fs:300-310 (28 bytes)."""
    _fields_ = [("X", C.c_float), ("Y", C.c_float), ("size", C.c_float), ("angle", C.c_float),
                ("response", C.c_float), ("octave", C.c_int), ("class_id", C.c_int)]


class DetectorResult(C.Structure):
    """MiniCVNative.h:23-29 / OpenCV.fs:329-337."""
    _fields_ = [("PointCount", C.c_int), ("DescriptorEntries", C.c_int), ("DescriptorElementType", C.c_int),
                ("Points", C.c_void_p), ("Descriptors", C.c_void_p)]


class MatchConfig(C.Structure):
    _fields_ = [("ratio", C.c_float), ("crossCheck", C.c_int), ("maxDistance", C.c_float), ("model", C.c_int)]


class ReplayState(C.Structure):
    _fields_ = [("niters", C.c_int64), ("bestIndex", C.c_int64), ("bestCount", C.c_int32),
                ("stopped", C.c_int32)]


METHOD_LSQ = 0
METHOD_RANSAC = 8
FLAG_FIXED_ITERS = 1
FLAG_NO_REFINE = 2
FLAG_FUSED_ERROR = 64   # bit 4 is retired (rejected by the library)
FLAG_CV_SAMPLER = 32    # OpenCV's own sample stream (cv::RNG(-1) + getSubset)
FLAG_SEVEN_POINT = 8
FLAG_FAST_MINIMAL = 16
FERR_SAMPSON = 0
FERR_EPIPOLAR = 1
MODEL_HOMOGRAPHY = 0
MODEL_FUNDAMENTAL = 1
MODEL_ESSENTIAL = 2
MODEL_PNP = 3
E_SLOTS = 10

_P = C.c_void_p
_I = C.c_int
_I64 = C.c_int64
_U64 = C.c_uint64
_D = C.c_double
_F = C.c_float

# name -> (restype, argtypes). Pointers are passed as void* (numpy .ctypes.data / device ints).
SIGNATURES = {
    # existing reference exports (OpenCV.fs:343-382)
    "cvRecoverPose": (_I, [_P, _I, _P, _P, _P, _P, _P]),
    "cvRecoverPoses": (_I, [_P, _I, _P, _P, _P, _P, _P, _P]),
    "cvDetectFeatures": (_P, [_P, _I, _I, _I, _I, _P]),
    "cvFreeFeatures": (None, [_P]),
    "cvTest": (None, []),
    "cvFivePoint": (_I, [_P, _P, _P]),
    "cvSolvePnP": (_I, [_P, _P, _I, M33d, _P, _I, _P, _P]),
    "cvSolvePnPRansac": (_I, [_P, _P, _I, M33d, _P, _I, _I, _F, _D, _P, _P, _P, _P]),
    "cvRefinePnPLM": (None, [_P, _P, _I, M33d, _P, _P, _P]),
    "cvRefinePnPVVS": (None, [_P, _P, _I, M33d, _P, _P, _P]),
    "solveAp3p": (_I, [_P, _P] + [_D] * 19),
    "cvDetectQRCode": (_I, [_P, _I, _I, _I, _P, _P]),
    "cvDetectArucoMarkers": (_I, [_P, _I, _I, _I, _P, _P]),
    # new hot-path exports
    "cvFindHomography": (_I, [_P, _P, _I, _P, _P, _P]),
    "cvFindFundamentalMat": (_I, [_P, _P, _I, _P, _P, _P]),
    "cvFindEssentialMat": (_I, [_P, _P, _I, _D, V2d, _P, _P, _P]),
    "cvSolvePnPRansacCfg": (_I, [_P, _P, _I, M33d, _P, _P, _P, _P, _P, _P]),
    "cvMatchFeatures": (_I, [_P, _P, _P, _P, _P, _I]),
    "cvMatchAndFindModel": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _P]),
    "cvMatchHamming": (_I, [_P, _I, _P, _I, _I, _P, _P, _P, _P]),
    "cvMatchL2": (_I, [_P, _I, _P, _I, _I, _P, _P, _P, _P]),
    "cvMatchHammingMulti": (_I, [_P, _I, _P, _I, _I, _I, _P, _P, _P, _P]),
    "cvMatchL2Multi": (_I, [_P, _I, _P, _I, _I, _I, _P, _P, _P, _P]),
    "cvFindScaledPose": (_I, [_D, _P, _P, _P, _I, _P, _P, _P, _P]),
    "cvFindScaledPoseCosts": (_I, [_P, _P, _P, _I, _P, _P, _P, _P]),
    "mcvGetLastError": (C.c_char_p, []),
    "mcvDeviceCount": (_I, []),
    "mcvVersion": (C.c_char_p, []),
    "mcvAbiVersion": (_I, []),
    "mcvCvSubsets": (_I64, [_I, _I, _P, _I, _I64, _P]),
    # device-level API
    "mcvRansacPlanCreate": (_P, [_I, _I, _I64]),
    "mcvRansacPlanDestroy": (None, [_P]),
    "mcvPackCorrespondences": (_I, [_P, _P, _I, _P, _P]),
    "mcvPackEssential": (_I, [_P, _P, _I, _D, V2d, _P, _P]),
    "mcvPackPnP": (_I, [_P, _P, _I, _P, _P]),
    "mcvRansacPlanSetCamera": (_I, [_P, _P, _P]),
    "mcvRansacEvaluate": (_I, [_P, _P, _I, _P, _I64, _I64, _P, _P, _P]),
    "mcvRansacFinalize": (_I, [_P, _P, _I, _P, _I64, _P, _P, _P]),
    "mcvReplayInit": (None, [_P, _I]),
    "mcvL2LastExactScans": (_I, []),
    "mcvL2LastGemmForm": (_I, []),
    "mcvReplayChunk": (_I, [_P, _P, _I64, _I64, _I, _I, _D, _I]),
    "mcvReplayChunkModels": (_I, [_P, _P, _I64, _I64, _I, _I, _I, _D, _I]),
    "mcvMatchHammingDevice": (_I, [_P, _I, _P, _I, _I, _P, _P, _P, _P, _P]),
    "mcvMatchHammingDeviceForm": (_I, [_P, _I, _P, _I, _I, _P, _P, _P, _P, _I, _P]),
    "mcvMatchL2Device": (_I, [_P, _I, _P, _I, _I, _P, _P, _P, _P, _P]),
    "mcvFindScaledPoseDevice": (_I, [_P, _P, _P, _I, _P, _P, _P, _P, _P]),
    "mcvProfileEnable": (None, [_I]),
    "mcvProfileReset": (None, []),
    "mcvProfileRead": (_I, [C.c_char_p, _P]),
    # test hooks
    "mcvHostHypothesis": (_I, [_I, _P, _I, _U64, _I64, _P, _P, _P]),
    "mcvHostPhilox": (None, [C.c_uint32] * 6 + [_P]),
    "mcvHostFingerprint": (_U64, [_P, C.c_size_t]),
    "mcvHostGlibcMath": (_I, [_I, _P, _P, _I, _P]),
    "mcvTestFingerprint": (_I, [_P, C.c_size_t, _P]),
    "mcvTestEigLogCap": (_I, [_I]),
    "mcvHostEssential": (_I, [_P, _I, _U64, _I64, _P, _P]),
    "mcvHostEssentialFast": (_I, [_P, _I, _U64, _I64, _P, _P]),
    "mcvHostFivePoint": (_I, [_P, _P]),
    "mcvHostFivePointRef": (_I, [_P, _P]),
    "mcvHostF7": (_I, [_P, _I, _U64, _I64, _P, _P]),
    "mcvHostDecomposeEssential": (None, [_P, _P, _P, _P]),
    "mcvHostRealRoots": (_I, [_P, _I, _I, _P]),
    "mcvHostPnP": (_I, [_P, _I, _P, _U64, _I64, _P, _P, _P]),
    "mcvHostPnPFast": (_I, [_P, _I, _P, _U64, _I64, _P, _P, _P]),
    "mcvHostPnPEpnp": (_I, [_P, _I, _P, _U64, _I64, _P, _P, _P]),
    "mcvHostPnpCert": (_I, [_P, _I, _P, _P, _P, C.c_float, _I, _P, _P]),
    "mcvHostSampsonCert": (_I, [_P, _I, _P, C.c_float, _I, _P, _P]),
    "mcvHostSqpnp": (_I, [_P, _P, _I, _P, _P, _P]),
    "mcvTestPnpSweep": (_I, [_P, _I, _P, _P, _I, C.c_float, _I, _I, _P]),
    "mcvHostEpnp5": (None, [_P, _P, _P, _P, _P]),
    "mcvHostSolveAp3p": (_I, [_P, _P, _P, _D, _D, _D, _D, _P, _P]),
    "mcvTestPnpHypotheses": (_I, [_P, _I, _P, _U64, _I64, _I, _I, _P, _P]),
    "mcvHostRodrigues": (None, [_P, _P, _P]),
    "mcvHostRodriguesInv": (None, [_P, _P]),
    "mcvTestRcpExhaustive": (C.c_longlong, [_I, _P]),
    "mcvTestDivF64": (C.c_longlong, [_I, C.c_ulonglong, C.c_longlong, _P]),
    "mcvTestHomographySweep": (_I, [_P, _I, _P, _I, _F, _I, _P]),
    "mcvHostScaledCosts": (_I, [_P, _P, _P, _I, _P, _P, _P, _P]),
}

_lib = None


def lib() -> C.CDLL:
    """Load libMiniCVNative.so (raises if it has not been built: no fallback)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(f"libMiniCVNative.so not found at {LIB_PATH}; run __graft_entry__.build()")
        # torch bundles its own libamdhip64.so.7 / libhsa-runtime64.so.1 (same SONAMEs as /opt/rocm's).
        # Whichever process-wide copy loads first serves both; if ours loaded first, torch would bring
        # a second HIP/HSA runtime whose device init fails. So let torch's copy load first when present.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    e = lib().mcvGetLastError()
    return e.decode() if e else ""


class NativeError(RuntimeError):
    pass


def check(ok: bool, what: str) -> None:
    if not ok:
        raise NativeError(f"{what}: {last_error()}")
