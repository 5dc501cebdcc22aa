"""Per-rank L2 step time of bench.py's query-sharded cfg5 (nq / N queries x 50k train x 128) for
N = 1, 2, 4, 8 on one GPU: what each rank of the driver's scaling run computes (device arrays;
`ms` = median of 10 synchronous calls, `async_ms` = 30 calls back to back / 30, as bench.py's timed
loop runs them)."""
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from minicv_amd import device as D, synthetic as S


def main():
    dev = torch.device("cuda:0")
    q, t, _ = S.l2_problem(50_000, 50_000, dim=128, seed=5)
    qd, td = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
    for n in (1, 2, 4, 8):
        cnt = (50_000 + n - 1) // n
        qs = qd[:cnt].contiguous()
        idx = torch.empty(cnt, dtype=torch.int32, device=dev)
        idx2 = torch.empty_like(idx)
        d1 = torch.empty(cnt, dtype=torch.float32, device=dev)
        d2 = torch.empty_like(d1)
        ts = []
        for k in range(13):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            D.match_l2(qs, td, idx, d1, idx2, d2)
            torch.cuda.synchronize()
            if k >= 3:
                ts.append(time.perf_counter() - t0)
        ms = float(np.median(ts)) * 1e3
        # back to back, as bench.py's timed loop runs a rank's steps (no synchronisation per step)
        steps = 30
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            D.match_l2(qs, td, idx, d1, idx2, d2)
        torch.cuda.synchronize()
        ams = (time.perf_counter() - t0) / steps * 1e3
        print(json.dumps({"ranks": n, "queries_per_rank": cnt, "ms": round(ms, 3), "async_ms": round(ams, 3),
                          "tflops_per_rank": round(2 * cnt * 50_000 * 128 / (ms * 1e-3) / 1e12, 1)}), flush=True)


if __name__ == "__main__":
    main()
