"""The 8-rank L2 share (6250 of cfg5's 50k queries x 50k train, 128-d) called 30 times back to back, for
rocprofv3 --kernel-trace --stats (per-kernel times of the share)."""
import sys

import torch

sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[2]))
from minicv_amd import device as D, synthetic as S

dev = torch.device("cuda:0")
cnt = int(sys.argv[1]) if len(sys.argv) > 1 else 6250
q, t, _ = S.l2_problem(50_000, 50_000, dim=128, seed=5)
qd, td = torch.from_numpy(q[:cnt]).to(dev), torch.from_numpy(t).to(dev)
idx = torch.empty(cnt, dtype=torch.int32, device=dev)
idx2 = torch.empty_like(idx)
d1 = torch.empty(cnt, dtype=torch.float32, device=dev)
d2 = torch.empty_like(d1)
for _ in range(30):
    D.match_l2(qd, td, idx, d1, idx2, d2)
torch.cuda.synchronize()
print("ok", cnt)
from minicv_amd import native as NL
print("queued exact scans", NL.lib().mcvL2LastExactScans())
