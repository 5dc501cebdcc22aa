"""Screen: L2 variants selected by mcvScreenSet(v) (screen builds only) at the 8 / 4-rank shares and the
full cfg5 call: outputs compared with variant 0, ms per call (10 back-to-back calls, median of 5)."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[2]))
from minicv_amd import device as D, native as NL, synthetic as S

dev = torch.device("cuda:0")
vs = [int(v) for v in sys.argv[1:]] or [0, 2]
q, t, _ = S.l2_problem(50_000, 50_000, dim=128, seed=5)
td = torch.from_numpy(t).to(dev)
for cnt in (6250, 12500, 50_000):
    qs = torch.from_numpy(q[:cnt]).to(dev)
    o = [torch.empty(cnt, dtype=torch.int32, device=dev), torch.empty(cnt, device=dev),
         torch.empty(cnt, dtype=torch.int32, device=dev), torch.empty(cnt, device=dev)]
    NL.lib().mcvScreenSet(0)
    D.match_l2(qs, td, o[0], o[1], o[2], o[3])
    torch.cuda.synchronize()
    ref = [x.cpu().clone() for x in o]
    for v in vs * 3:
        NL.lib().mcvScreenSet(v)
        for _ in range(3):
            D.match_l2(qs, td, o[0], o[1], o[2], o[3])
        torch.cuda.synchronize()
        same = all(torch.equal(a.cpu(), b) for a, b in zip(o, ref))
        ts = []
        for k in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                D.match_l2(qs, td, o[0], o[1], o[2], o[3])
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) / 10)
        print(json.dumps({"v": v, "nq": cnt, "ms": round(float(np.median(ts)) * 1e3, 4), "same": same}), flush=True)
NL.lib().mcvScreenSet(0)
