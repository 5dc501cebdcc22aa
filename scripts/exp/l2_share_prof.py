"""One rank's L2 share (50k / N queries x 50k train x 128) called back to back, for a rocprofv3
kernel trace of what the N-GPU step is made of. Usage: l2_share_prof.py N"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))


def main():
    import torch
    from minicv_amd import device as D, synthetic as S
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device("cuda:0")
    q, t, _ = S.l2_problem(50_000, 50_000, dim=128, seed=5)
    cnt = (50_000 + n - 1) // n
    qs, td = torch.from_numpy(q[:cnt]).to(dev), torch.from_numpy(t).to(dev)
    idx, idx2 = (torch.empty(cnt, dtype=torch.int32, device=dev) for _ in range(2))
    d1, d2 = (torch.empty(cnt, dtype=torch.float32, device=dev) for _ in range(2))
    for _ in range(3):
        D.match_l2(qs, td, idx, d1, idx2, d2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        D.match_l2(qs, td, idx, d1, idx2, d2)
    torch.cuda.synchronize()
    print(f"N={n} share {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms per call", flush=True)


if __name__ == "__main__":
    main()
