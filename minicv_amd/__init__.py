"""minicv_amd — MI355X-native (gfx950) drop-in for MiniCV's matching + RANSAC hot path.

The product is libMiniCVNative.so (C-ABI, include/minicv_native.h), built from csrc/ by
minicv_amd.build. This package is the host-side mirror of the reference's managed wrappers
(opencv.py, camera.py), a device-level API for HBM-resident inputs (device.py) and synthetic
workloads.
"""
from . import native
from .native import RansacConfig, NativeError
from .opencv import RansacParams, findHomography, findFundamentalMat, matchHamming, matchL2, recoverPose
from . import camera
from .camera import Camera, CameraPose, findScaled

__all__ = ["native", "RansacConfig", "NativeError", "RansacParams", "findHomography", "findFundamentalMat",
           "matchHamming", "matchL2", "recoverPose", "camera", "Camera", "CameraPose", "findScaled"]
