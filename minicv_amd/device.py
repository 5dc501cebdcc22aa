"""Device-level API over torch-allocated HBM buffers (bench.py, multi-GPU ranks).

PyTorch only provides device memory, streams and torch.distributed (RCCL); every kernel runs in
libMiniCVNative.so. Pointers cross the C-ABI as plain integers (tensor.data_ptr()) and the
stream as the raw hipStream_t handle of torch's current stream.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import native as N


def _stream_handle(stream=None) -> int:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


class RansacPlan:
    """Workspace for one RANSAC problem family on the current device."""

    def __init__(self, model: int, max_n: int, max_hyps: int):
        self.model = model
        self._p = N.lib().mcvRansacPlanCreate(model, int(max_n), int(max_hyps))
        N.check(bool(self._p), "mcvRansacPlanCreate")

    def set_camera(self, K, dist=None) -> None:
        """PnP plans: camera matrix (3x3) and distortion (k1, k2, p1, p2)."""
        K9 = np.ascontiguousarray(np.asarray(K, dtype=np.float64).ravel())
        d = None if dist is None else np.ascontiguousarray(np.asarray(dist, dtype=np.float64))
        ok = N.lib().mcvRansacPlanSetCamera(self._p, K9.ctypes.data, None if d is None else d.ctypes.data)
        N.check(ok == 1, "mcvRansacPlanSetCamera")

    def close(self):
        if self._p:
            N.lib().mcvRansacPlanDestroy(self._p)
            self._p = None

    __del__ = close

    def evaluate(self, pts4, n: int, cfg: N.RansacConfig, hyp_begin: int, hyp_count: int, key, counts=None,
                 stream=None) -> None:
        """Asynchronous: best packed key of [hyp_begin, hyp_begin + hyp_count) -> key[0] (int64 tensor),
        first sampler failure -> key[1]."""
        ok = N.lib().mcvRansacEvaluate(self._p, pts4.data_ptr(), int(n), C.addressof(cfg), int(hyp_begin),
                                       int(hyp_count), key.data_ptr(),
                                       counts.data_ptr() if counts is not None else None, _stream_handle(stream))
        N.check(ok == 1, "mcvRansacEvaluate")

    def finalize(self, pts4, n: int, cfg: N.RansacConfig, hyp: int, mask, stream=None):
        """-> (inlier count, model 3x3 float64); writes the uint8 mask tensor. Synchronises the stream."""
        m = (C.c_double * 9)()
        cnt = N.lib().mcvRansacFinalize(self._p, pts4.data_ptr(), int(n), C.addressof(cfg), int(hyp), m,
                                        mask.data_ptr(), _stream_handle(stream))
        N.check(cnt > 0, "mcvRansacFinalize")
        return cnt, np.array(m[:], dtype=np.float64).reshape(3, 3)


def unpack_key(key: int):
    """(count, hypothesis index) from the packed key (count << 32 | 0xFFFFFFFF - idx); (0, -1) if none."""
    key = int(key) & 0xFFFFFFFFFFFFFFFF
    if key == 0:
        return 0, -1
    return key >> 32, 0xFFFFFFFF - (key & 0xFFFFFFFF)


def pack_points_tensor(src: np.ndarray, dst: np.ndarray, device):
    """(N,2)+(N,2) fp64 -> device float32 [N,4] {x, y, x', y'} (float cast as convertTo(CV_32F))."""
    import torch
    p = np.concatenate([src, dst], axis=1).astype(np.float32)
    return torch.from_numpy(np.ascontiguousarray(p)).to(device)


HAMMING_FORMS = {"gemm": 0, "popcount": 1}


def match_hamming(q, t, idx, dist, idx2=None, dist2=None, stream=None, form="gemm") -> None:
    """form: "gemm" (fp4 GEMM on the matrix cores, the default) or "popcount" (XOR / popcount sweep)."""
    r = N.lib().mcvMatchHammingDeviceForm(q.data_ptr(), q.shape[0], t.data_ptr(), t.shape[0], q.shape[1],
                                          idx.data_ptr(), dist.data_ptr(),
                                          idx2.data_ptr() if idx2 is not None else None,
                                          dist2.data_ptr() if dist2 is not None else None, HAMMING_FORMS[form],
                                          _stream_handle(stream))
    N.check(r == q.shape[0], "mcvMatchHammingDevice")


def match_l2(q, t, idx, dist, idx2=None, dist2=None, stream=None) -> None:
    r = N.lib().mcvMatchL2Device(q.data_ptr(), q.shape[0], t.data_ptr(), t.shape[0], q.shape[1],
                                 idx.data_ptr(), dist.data_ptr(),
                                 idx2.data_ptr() if idx2 is not None else None,
                                 dist2.data_ptr() if dist2 is not None else None, _stream_handle(stream))
    N.check(r == q.shape[0], "mcvMatchL2Device")


def pack_essential_tensor(a: np.ndarray, b: np.ndarray, focal: float, pp, device, stream=None):
    """(N,2)+(N,2) fp64 pixels -> device float64 [N,4] normalised (x - pp) / focal, computed on the GPU
    (mcvPackEssential; synchronises the stream)."""
    import torch
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    out = torch.empty((a.shape[0], 4), dtype=torch.float64, device=device)
    ok = N.lib().mcvPackEssential(a.ctypes.data, b.ctypes.data, a.shape[0], float(focal),
                                  N.V2d(float(pp[0]), float(pp[1])), out.data_ptr(), _stream_handle(stream))
    N.check(ok == 1, "mcvPackEssential")
    return out


def pack_pnp_tensor(img: np.ndarray, world: np.ndarray, device, stream=None):
    """(N,2) image + (N,3) world fp64 -> device PnpPoint [N][8] float32 (packed on the GPU)."""
    import torch
    img = np.ascontiguousarray(img, dtype=np.float64)
    world = np.ascontiguousarray(world, dtype=np.float64)
    out = torch.empty((img.shape[0], 8), dtype=torch.float32, device=device)
    ok = N.lib().mcvPackPnP(img.ctypes.data, world.ctypes.data, img.shape[0], out.data_ptr(), _stream_handle(stream))
    N.check(ok == 1, "mcvPackPnP")
    return out
