"""Probe (needs a screen build exporting mcvScreenStamps(ptr), a kernel argument the product lacks): per-wave s_memrealtime stamps of the fp4 Hamming GEMM —
entry, query block expanded, tile loop done (last segment), arrival add returned, fold done, exit
(100 MHz ticks) — for one call after 30 warm calls; raw arrays to gpurun_out/ham_stamps_<nq>.npy."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[2]))
from minicv_amd import device as D, native as NL, synthetic as S

dev = torch.device("cuda:0")
buf = torch.zeros(8192 * 8 * 8, dtype=torch.int64, device=dev)
for nq in (1250, 10_000):
    q, t, _ = S.hamming_problem(nq, 10_000, seed=2)
    qd, td = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
    o = [torch.empty(nq, dtype=torch.int32, device=dev) for _ in range(4)]
    for rep in range(3):
        for _ in range(30):
            D.match_hamming(qd, td, *o)
        torch.cuda.synchronize()
        buf.fill_(-1)
        NL.lib().mcvScreenStamps(ctypes.c_void_p(buf.data_ptr()))
        D.match_hamming(qd, td, *o)
        torch.cuda.synchronize()
        NL.lib().mcvScreenStamps(ctypes.c_void_p(0))
        a = buf.view(-1, 8).cpu().numpy()
        a = a[a[:, 0] != -1]
        np.save(f"gpurun_out/ham_stamps_{nq}_{rep}.npy", a)
        t0 = a[:, 0].min()
        rel = lambda c: (a[:, c] - t0) / 100.0
        print(nq, rep, "waves", len(a), " ".join(
            f"{n}: {np.min(rel(c)):.1f}/{np.median(rel(c)):.1f}/{np.max(rel(c)):.1f}"
            for n, c in [("entry", 0), ("expanded", 1), ("loop", 2), ("arrived", 3), ("exit", 5)]), flush=True)
