"""Debug: cfg2 Hamming GEMM form vs the oracle, per array, for the current MCV_HAMMING_* settings."""
import os
import sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
from minicv_amd import opencv, synthetic as S
import _oracle as O
q, t, _ = S.hamming_problem(10_000, 10_000, seed=2)
ref = O.match_hamming(q, t)
for trial in range(3):
    got = opencv.matchHamming(q, t)
    for name, g, r in zip(["idx", "dist", "idx2", "dist2"], got, ref):
        bad = np.nonzero(g != r)[0]
        if len(bad):
            i = bad[0]
            print(trial, name, "mismatches", len(bad), "first q", i, "got", [a[i] for a in got], "ref", [a[i] for a in ref])
print("done", os.environ.get("MCV_HAMMING_SUB"), os.environ.get("MCV_HAMMING_QT"))
