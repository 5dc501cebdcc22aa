"""Screen: Hamming GEMM variants selected by mcvScreenSet(v) (screen builds only): outputs compared with
variant 0, per-call time over 200 calls, alternating variants, at the rank-share query counts."""
import json
import sys

import torch

sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[2]))
from minicv_amd import device as D, native as NL, synthetic as S

dev = torch.device("cuda:0")
vs = [int(v) for v in sys.argv[1:]] or [0, 1]
for nq, nt in [(1250, 10_000), (5000, 10_000), (10_000, 10_000), (10_000, 40_000)]:
    q, t, _ = S.hamming_problem(nq, nt, seed=2)
    qd, td = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
    o = [torch.empty(nq, dtype=torch.int32, device=dev) for _ in range(4)]
    NL.lib().mcvScreenSet(0)
    D.match_hamming(qd, td, *o)
    torch.cuda.synchronize()
    ref = torch.stack(o).cpu()
    for v in vs * 3:
        NL.lib().mcvScreenSet(v)
        for _ in range(20):
            D.match_hamming(qd, td, *o)
        torch.cuda.synchronize()
        same = bool(torch.equal(torch.stack(o).cpu(), ref))
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(200):
            D.match_hamming(qd, td, *o)
        b.record()
        torch.cuda.synchronize()
        print(json.dumps({"v": v, "nq": nq, "nt": nt, "us": round(a.elapsed_time(b) / 200 * 1e3, 2), "same": same}),
              flush=True)
NL.lib().mcvScreenSet(0)
