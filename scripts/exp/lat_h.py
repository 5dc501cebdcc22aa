"""Experiment: per-call timeline of cvFindHomography at n=500 (kernels + HIP API), 10 calls."""
import sys
import time
sys.path.insert(0, '/root/repo')
import numpy as np
from minicv_amd import opencv, synthetic as S
src, dst, _ = S.homography_problem(500, 1)
for _ in range(3):
    opencv.findHomography(src, dst)
ts = []
for _ in range(10):
    t = time.perf_counter()
    opencv.findHomography(src, dst)
    ts.append(time.perf_counter() - t)
print("median ms", np.median(ts) * 1e3)
