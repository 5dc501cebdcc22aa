"""Host mirror of the reference's camera / pose records and CameraPose.findScaled
(/root/reference/src/MiniCV/Camera.fs, /root/reference/src/MiniCV/CameraPose.fs).

`findScaled` keeps the F# signature and semantics (CameraPose.fs:39-134): the O(N^2) scale
hypothesize-and-verify runs in libMiniCVNative.so on the GPU (cvFindScaledPose); this module only
marshals the records and builds the scaled pose, as the F# wrapper would. The
numpy helpers below (lookAt, project1, transformed_view) build test/bench inputs; they are not on
the product path.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field

import numpy as np

from . import native as N


def _v3(a) -> np.ndarray:
    return np.asarray(a, np.float64).reshape(3)


@dataclass
class Camera:
    """Camera.fs:7-14 (location, forward, up, right, focal)."""
    location: np.ndarray
    forward: np.ndarray
    up: np.ndarray
    right: np.ndarray
    focal: np.ndarray

    def to_c(self) -> N.Camera:
        c = N.Camera()
        for name in ("location", "forward", "up", "right"):
            v = _v3(getattr(self, name))
            setattr(c, name, N.V3d(*v))
        f = np.asarray(self.focal, np.float64).reshape(2)
        c.focal = N.V2d(f[0], f[1])
        return c


def lookAt(eye, center, sky, f) -> Camera:
    """Camera.lookAt (Camera.fs:93-104)."""
    eye, center, sky = _v3(eye), _v3(center), _v3(sky)
    fw = center - eye
    fw = fw / np.linalg.norm(fw)
    r = np.cross(fw, sky)
    r = r / np.linalg.norm(r)
    u = np.cross(r, fw)
    u = u / np.linalg.norm(u)
    return Camera(eye, fw, u, r, np.asarray(f, np.float64).reshape(2))


def project1(c: Camera, pts: np.ndarray):
    """Camera.project1 (Camera.fs:72-83), vectorised: (c[n, 2], visible[n])."""
    o = np.asarray(pts, np.float64).reshape(-1, 3) - c.location
    pc = np.stack([o @ c.right, o @ c.up, o @ c.forward], axis=1)
    xy = c.focal * pc[:, :2] / pc[:, 2:3]
    vis = (pc[:, 2] >= 0) & np.all(xy >= -1.0, axis=1) & np.all(xy <= 1.0, axis=1)
    return xy, vis


@dataclass
class CameraPose:
    """CameraPose.fs:7-16 (struct: the default value is all zero)."""
    RotationIndex: int = 0
    ScaleSign: int = 0
    Rotation: np.ndarray = field(default_factory=lambda: np.zeros((3, 3)))
    Translation: np.ndarray = field(default_factory=lambda: np.zeros(3))
    IsInverse: bool = False


def _sign(f: float) -> int:
    if math.isnan(f):   # F# `sign nan` throws (System.Math.Sign)
        raise ArithmeticError("sign of NaN")
    return int(f > 0) - int(f < 0)


def scale(f: float, pose: CameraPose) -> CameraPose:
    """CameraPose.scale (CameraPose.fs:31-33)."""
    return CameraPose(pose.RotationIndex, _sign(f) * pose.ScaleSign, pose.Rotation, f * _v3(pose.Translation),
                      pose.IsInverse)


def transformation(pose: CameraPose) -> np.ndarray:
    """CameraPose.transformation (CameraPose.fs:24-29): 4x4 forward matrix [R | R t]."""
    m = np.eye(4)
    R = np.asarray(pose.Rotation, np.float64).reshape(3, 3)
    m[:3, :3] = R
    m[:3, 3] = R @ _v3(pose.Translation)
    return m


def transformed_view(t: np.ndarray, c: Camera) -> Camera:
    """Camera.transformedView (Camera.fs:60-70) with a 4x4 forward matrix."""
    to_world = np.eye(4)
    to_world[:3, 0], to_world[:3, 1], to_world[:3, 2], to_world[:3, 3] = c.right, c.up, -c.forward, c.location
    m = to_world @ t
    nz = lambda v: v / np.linalg.norm(v)
    return Camera(m[:3, 3].copy(), nz(-m[:3, 2]), nz(m[:3, 1]), nz(m[:3, 0]), np.asarray(c.focal, np.float64))


def _split_observations(worldObservations):
    if isinstance(worldObservations, tuple) and len(worldObservations) == 2 and \
            isinstance(worldObservations[0], np.ndarray):
        world, obs = worldObservations
    else:
        pairs = list(worldObservations)
        world = np.array([p[0] for p in pairs], np.float64).reshape(-1, 3)
        obs = np.array([p[1] for p in pairs], np.float64).reshape(-1, 2)
    return (np.ascontiguousarray(world, np.float64).reshape(-1, 3),
            np.ascontiguousarray(obs, np.float64).reshape(-1, 2))


def findScaled(inlierThreshold: float, srcCam: Camera, worldObservations, pose: CameraPose):
    """CameraPose.findScaled (CameraPose.fs:39-134) -> (cost, scaled pose).

    worldObservations: a sequence of (V3d, V2d) pairs (the F# list) or a (world[n,3], obs[n,2])
    tuple of arrays. Raises RuntimeError when the native call fails (no CPU fallback)."""
    world, obs = _split_observations(worldObservations)
    n = world.shape[0]
    if n == 0:   # CameraPose.fs:42
        return math.inf, CameraPose()
    R = N.M33d()
    R.M[:] = np.asarray(pose.Rotation, np.float64).reshape(9)
    t = N.V3d(*_v3(pose.Translation))
    cost, s = C.c_double(0), C.c_double(0)
    cam = srcCam.to_c()
    k = N.lib().cvFindScaledPose(float(inlierThreshold), C.addressof(cam), world.ctypes.data, obs.ctypes.data, n,
                                 C.addressof(R), C.addressof(t), C.addressof(cost), C.addressof(s))
    if k < 0:
        raise RuntimeError(f"cvFindScaledPose failed: {N.last_error()}")
    return cost.value, scale(s.value, pose)


def findScaledCosts(srcCam: Camera, world: np.ndarray, obs: np.ndarray, pose: CameraPose):
    """Per-candidate (scales[2n], costs[2n]) of findScaled, in candidate order (analysis helper)."""
    world = np.ascontiguousarray(world, np.float64).reshape(-1, 3)
    obs = np.ascontiguousarray(obs, np.float64).reshape(-1, 2)
    n = world.shape[0]
    R = N.M33d()
    R.M[:] = np.asarray(pose.Rotation, np.float64).reshape(9)
    t = N.V3d(*_v3(pose.Translation))
    sc, co = np.empty(2 * n), np.empty(2 * n)
    cam = srcCam.to_c()
    if N.lib().cvFindScaledPoseCosts(C.addressof(cam), world.ctypes.data, obs.ctypes.data, n, C.addressof(R),
                                     C.addressof(t), sc.ctypes.data, co.ctypes.data) < 0:
        raise RuntimeError(f"cvFindScaledPoseCosts failed: {N.last_error()}")
    return sc, co
