"""cfg2 Hamming step anatomy: host time per call (no sync), wall time per call with / without the
profiling events, for both kernel forms. Run on the GPU box (optionally under rocprofv3 --kernel-trace)."""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from minicv_amd import device as D, native as NL, synthetic as S  # noqa: E402

dev = torch.device("cuda:0")
q, t, _ = S.hamming_problem(10_000, 10_000, seed=2)
qd, td = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
idx, dist, idx2, dist2 = (torch.empty(10_000, dtype=torch.int32, device=dev) for _ in range(4))
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
for form in ("gemm", "popcount"):
    for prof in (0, 1):
        for _ in range(10):
            D.match_hamming(qd, td, idx, dist, idx2, dist2, form=form)
        torch.cuda.synchronize()
        NL.lib().mcvProfileReset()
        NL.lib().mcvProfileEnable(prof)
        t0 = time.perf_counter()
        for _ in range(steps):
            D.match_hamming(qd, td, idx, dist, idx2, dist2, form=form)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        NL.lib().mcvProfileEnable(0)
        print(f"{form:8s} prof={prof}: host {1e6 * (t1 - t0) / steps:.1f} us/call, wall {1e6 * (t2 - t0) / steps:.1f} us/step",
              flush=True)
