import sys, time
sys.path.insert(0, '/root/repo')
import numpy as np
from minicv_amd import opencv, synthetic as S
a, b, *_ = S.essential_problem(500, seed=2)
cfg = opencv.recoverPoseConfig(800.0, (640.0, 360.0), 0.999, 1.0)
for _ in range(5):
    opencv.recoverPose(cfg, a, b)
a5, b5, *_ = S.essential_problem(5, seed=6, outlier_frac=0)
for _ in range(5):
    opencv.fivepoint(a5, b5)
