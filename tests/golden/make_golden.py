"""Regenerate the committed golden fixtures (run from the repo root: python tests/golden/make_golden.py).

Inputs are the seeded synthetic workloads of minicv_amd/synthetic.py at sizes the oracle finishes
in well under a second; expected outputs come from oracle/oracle.c after it passed its own
known-answer tests (tests/test_oracle.py). The reference itself cannot produce vectors here
(OpenCV absent), so these fixtures pin regressions of both the oracle and the
GPU path, not OpenCV parity.
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import _oracle as O  # noqa: E402
from minicv_amd import synthetic as S  # noqa: E402

OUT = Path(__file__).resolve().parent


def cfg1():
    src, dst, _ = S.homography_problem(200, 1)
    thr, conf, iters, seed = 5e-3, 0.995, 2000, 1
    cnt, H, mask, best = O.find_homography(src, dst, thr=thr, conf=conf, max_iters=iters, seed=seed)
    pts4 = O.pack4(src, dst)
    counts = O.h_counts(pts4, seed, 0, 256, float(np.float32(thr * thr)))
    np.savez_compressed(OUT / "cfg1_homography.npz", src=src, dst=dst, thr=thr, conf=conf, max_iters=iters,
                        seed=seed, count=cnt, H=H, mask=mask, best_hyp=best, counts=counts)


def hypotheses():
    src, dst, _ = S.homography_problem(40, 21, outlier_frac=0.3)
    pts4 = O.pack4(src, dst)
    seed, hyps = 0xDEADBEEF12345678, np.arange(0, 96, dtype=np.int64) * 977
    rows = [O.h_hypothesis(pts4, seed, int(h)) for h in hyps]
    np.savez_compressed(OUT / "hypotheses.npz", pts4=pts4, seed=np.uint64(seed), hyps=hyps,
                        status=np.array([r[0] for r in rows], dtype=np.int32), H=np.stack([r[1] for r in rows]),
                        hf=np.stack([r[2] for r in rows]), idx=np.stack([r[3] for r in rows]))


def matchers():
    hq, ht, _ = S.hamming_problem(256, 512, seed=2)
    h = O.match_hamming(hq, ht)
    lq, lt, _ = S.l2_problem(128, 256, dim=128, seed=5)
    l = O.match_l2(lq, lt)
    np.savez_compressed(OUT / "matchers.npz", hq=hq, ht=ht, h_idx=h[0], h_dist=h[1], h_idx2=h[2], h_dist2=h[3],
                        lq=lq, lt=lt, l_idx=l[0], l_dist=l[1], l_idx2=l[2], l_dist2=l[3])


def fundamental():
    a, b, _, _ = S.fundamental_problem(500, 4)
    thr, conf, iters, seed = 5e-3, 0.99, 1000, 4
    cnt, F, mask, best = O.find_fundamental(a, b, thr=thr, conf=conf, max_iters=iters, seed=seed)
    np.savez_compressed(OUT / "fundamental.npz", a=a, b=b, thr=thr, conf=conf, max_iters=iters, seed=seed,
                        count=cnt, F=F, mask=mask, best_hyp=best)


if __name__ == "__main__":
    fundamental()
    cfg1()
    hypotheses()
    matchers()
    print("golden fixtures written to", OUT)
