"""What one rank of the driver's 1/2/4/8-GPU run computes, timed on one GPU.

For the strong-scaling workloads (fundamental, essential, pnp: a fixed 2^20-hypothesis call sharded
over the ranks; l2: 50k queries sharded) rank r of N evaluates 1/N of the work, so the N-GPU step
time is this share's one-GPU step time plus the exchange (one 16-byte all-reduce per call for the
RANSAC workloads, none for the matchers). The predicted speed-up at N ranks is t(1) / t(1/N).
Homography is weak scaling (2^20 hypotheses per GPU): its share is the full step at every N.

Runs bench.py at world size 1 with `--hyps total / N` (its per-GPU hypothesis count) and the L2
query shards directly; one JSON line per (workload, N) plus a summary line per workload.
"""
import json
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
TOTAL = 1 << 20
RANKS = (1, 2, 4, 8)


def bench_share(workload: str, hyps: int, steps: int) -> float:
    cmd = [sys.executable, "-u", str(ROOT / "bench.py"), "--workload", workload, "--hyps", str(hyps),
           "--steps", str(steps), "--warmup", "2", "--no-cpu-baseline", "--no-secondary"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, check=True).stdout
    line = next(json.loads(l) for l in out.splitlines() if l.startswith("{"))
    return float(line["ms_per_step"])


def l2_shares():
    import torch
    from minicv_amd import device as D, synthetic as S
    dev = torch.device("cuda:0")
    q, t, _ = S.l2_problem(50_000, 50_000, dim=128, seed=5)
    qd, td = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
    res = {}
    for n in RANKS:
        cnt = (50_000 + n - 1) // n
        qs = qd[:cnt].contiguous()
        idx = torch.empty(cnt, dtype=torch.int32, device=dev)
        idx2 = torch.empty_like(idx)
        d1 = torch.empty(cnt, dtype=torch.float32, device=dev)
        d2 = torch.empty_like(d1)
        # as bench.py's step loop: calls back to back on the stream, one synchronize per timed run (a
        # synchronize per call would add the host round trip to a 0.3 ms share)
        for _ in range(3):
            D.match_l2(qs, td, idx, d1, idx2, d2)
        ts = []
        for k in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                D.match_l2(qs, td, idx, d1, idx2, d2)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) / 10)
        res[n] = float(np.median(ts)) * 1e3
    return res


def main():
    which = sys.argv[1:] or ["fundamental", "essential", "pnp", "l2"]
    for w in which:
        if w == "l2":
            ms = l2_shares()
        else:
            ms = {}
            for n in RANKS:
                ms[n] = bench_share(w, TOTAL // n, 4 if n == 1 else 6)
                print(json.dumps({"workload": w, "ranks": n, "hyps_per_rank": TOTAL // n,
                                  "ms_per_step": round(ms[n], 3)}), flush=True)
        pred = {n: round(ms[1] / ms[n], 2) for n in RANKS}
        print(json.dumps({"workload": w, "share_ms": {n: round(v, 3) for n, v in ms.items()},
                          "predicted_speedup": pred}), flush=True)


if __name__ == "__main__":
    main()
