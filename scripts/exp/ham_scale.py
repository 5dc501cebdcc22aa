"""Hamming GEMM form: per-call time vs problem size (fixed vs per-tile cost), cfg2 shapes and multiples."""
import json
import sys

import torch

sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[2]))
from minicv_amd import device as D, synthetic as S

dev = torch.device("cuda:0")
for nq, nt in [(10_000, 10_000), (10_000, 20_000), (10_000, 40_000), (20_000, 10_000), (40_000, 10_000),
               (5_000, 10_000), (2_500, 10_000), (10_000, 80_000)]:
    q, t, _ = S.hamming_problem(nq, nt, seed=2)
    qd, td = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
    o = [torch.empty(nq, dtype=torch.int32, device=dev) for _ in range(4)]
    for _ in range(10):
        D.match_hamming(qd, td, *o)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(200):
        D.match_hamming(qd, td, *o)
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / 200 * 1e3
    print(json.dumps({"nq": nq, "nt": nt, "us": round(us, 2), "Tops": round(2 * 256 * nq * nt / us / 1e6, 1)}), flush=True)
