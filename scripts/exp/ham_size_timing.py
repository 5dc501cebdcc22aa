"""Per-call time of cvMatchHamming (GEMM form) at the query counts of the 1/2/4/8-rank shares of cfg2
(10k queries x 10k train) and at 10k x 40k, 200 calls each, three repeats."""
import json
import sys

import torch

sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[2]))
from minicv_amd import device as D, synthetic as S

dev = torch.device("cuda:0")
for nq, nt in [(1250, 10_000), (2500, 10_000), (5000, 10_000), (10_000, 10_000), (10_000, 40_000)]:
    q, t, _ = S.hamming_problem(nq, nt, seed=2)
    qd, td = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
    o = [torch.empty(nq, dtype=torch.int32, device=dev) for _ in range(4)]
    us = []
    for rep in range(3):
        for _ in range(20):
            D.match_hamming(qd, td, *o)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(200):
            D.match_hamming(qd, td, *o)
        b.record()
        torch.cuda.synchronize()
        us.append(round(a.elapsed_time(b) / 200 * 1e3, 2))
    print(json.dumps({"nq": nq, "nt": nt, "us_per_call": us}), flush=True)
