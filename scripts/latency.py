#!/usr/bin/env python3
"""Per-call latency of the host-pointer exports at the sizes a MiniCV caller uses (the F# wrappers
call these synchronously with host arrays): median of 20 calls after 3 warm-ups, including the
H2D/D2H copies. Prints one JSON line per export."""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from minicv_amd import camera as CM, opencv, synthetic as S  # noqa: E402


def timed(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return float(np.median(ts)) * 1e3


def main():
    out = []
    for n in (500, 5000):
        src, dst, _ = S.homography_problem(n, 1)
        out.append(("cvFindHomography", n, timed(lambda: opencv.findHomography(src, dst))))
        a, b, *_ = S.essential_problem(n, seed=2)
        cfg = opencv.recoverPoseConfig(800.0, (640.0, 360.0), 0.999, 1.0)
        out.append(("cvRecoverPose", n, timed(lambda: opencv.recoverPose(cfg, a, b))))
        img, W, _, K, d, _, _ = S.pnp_problem(n, seed=3)
        out.append(("cvSolvePnPRansac", n, timed(lambda: opencv.solvePnPRansac(img, W, K, d, reproj_error=2.0))))
        img0, W0, _, K0, d0, _, _ = S.pnp_problem(n, seed=8, outlier_frac=0.0, sigma=0.5)
        out.append(("cvSolvePnP(SQPNP)", n, timed(lambda: opencv.solvePnP(img0, W0, K0, d0, kind="SQPNP"))))
        out.append(("cvSolvePnP(EPNP)", n, timed(lambda: opencv.solvePnP(img0, W0, K0, d0, kind="EPNP"))))
        fa, fb, _, _ = S.fundamental_problem(n, 4)
        out.append(("cvFindFundamentalMat", n, timed(lambda: opencv.findFundamentalMat(fa, fb))))
        q, t, _ = S.hamming_problem(n, n, seed=5)
        out.append(("cvMatchHamming", n, timed(lambda: opencv.matchHamming(q, t))))
        lq, lt, _ = S.l2_problem(n, n, dim=128, seed=9)
        out.append(("cvMatchL2", n, timed(lambda: opencv.matchL2(lq, lt))))
        cam, pose, W3, O2, _ = S.scaled_problem(n, seed=7)
        out.append(("cvFindScaledPose", n, timed(lambda: CM.findScaled(0.01, cam, (W3, O2), pose))))
    a, b, *_ = S.essential_problem(5, seed=6, outlier_frac=0)
    out.append(("cvFivePoint", 5, timed(lambda: opencv.fivepoint(a, b))))
    for name, n, ms in out:
        print(json.dumps({"export": name, "n": n, "median_ms": round(ms, 3)}), flush=True)


if __name__ == "__main__":
    main()
