"""Experiment: timelines of single host-API calls (10 each after warm-up) for rocprofv3 traces."""
import sys
sys.path.insert(0, '/root/repo')
from minicv_amd import opencv, synthetic as S
src, dst, _ = S.homography_problem(500, 1)
a, b, *_ = S.essential_problem(500, seed=2)
cfg = opencv.recoverPoseConfig(800.0, (640.0, 360.0), 0.999, 1.0)
img, W, _, K, d, _, _ = S.pnp_problem(500, seed=3)
for _ in range(3):
    opencv.findHomography(src, dst); opencv.recoverPose(cfg, a, b); opencv.solvePnPRansac(img, W, K, d, reproj_error=2.0)
for _ in range(10):
    opencv.findHomography(src, dst)
for _ in range(10):
    opencv.recoverPose(cfg, a, b)
for _ in range(10):
    opencv.solvePnPRansac(img, W, K, d, reproj_error=2.0)
