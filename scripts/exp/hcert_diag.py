"""Diagnostics of the certified homography sweep: fraction of hypotheses the sweep hands to the exact
redo pass (MCV_HCERT_NOREDO=1 leaves them marked -3), per variant."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.getcwd())
from minicv_amd import native as N, opencv, synthetic as S, device as D
n, H = 100_000, 1 << 16
src, dst, _ = S.homography_problem(n, 3)
dev = torch.device("cuda:0")
pts = D.pack_points_tensor(src, dst, dev)
plan = D.RansacPlan(N.MODEL_HOMOGRAPHY, n, H)
cfg = opencv.RansacParams(threshold=5e-3, seed=3, fixed_iters=True, max_iters=H).to_c()
key = torch.zeros(2, dtype=torch.int64, device=dev)
counts = torch.zeros(H, dtype=torch.int32, device=dev)
plan.evaluate(pts, n, cfg, 0, H, key, counts)
c = counts.cpu().numpy()
print(os.environ.get("MCV_HCERT_VARIANT"), "redo", int((c == -3).sum()), "of", H, "nomodel", int((c == -1).sum()),
      "max", int(c.max()), "sum", int(c[c >= 0].sum()))
