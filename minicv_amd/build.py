"""Build libMiniCVNative.so (the MI355X drop-in) with hipcc for gfx950.

Every source under csrc/ is compiled as HIP (`-x hip`), objects go to build/, and the shared
library lands where Aardvark's native loader looks for MiniCVNative
(libs/Native/MiniCV/linux/AMD64/, cf. /root/reference/src/MiniCVNative/CMakeLists.txt:33-34).

-ffp-contract=off is global on purpose: the RANSAC error and minimal solvers must round exactly
as written, on the GPU and in the host twin, for the inlier masks to be bit-exact.
-fno-slp-vectorize: keep f32 VALU ops single-lane; SLP packing into v_pk_*_f32 needs v_mov to
build operand pairs from scalar model coefficients and is an anti-lever beside the sweep's
SGPR-operand arithmetic (cdna_hip_programming.md, packed f32 VALU).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "minicv_amd" / "csrc"
INCLUDE = ROOT / "include"
BUILD = ROOT / "build" / "native"
LIBDIR = ROOT / "libs" / "Native" / "MiniCV" / "linux" / "AMD64"
LIB = LIBDIR / "libMiniCVNative.so"
ARCH = os.environ.get("MCV_OFFLOAD_ARCH", "gfx950")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = [
    "-x", "hip", "-std=c++17", "-O3", "-fPIC", f"--offload-arch={ARCH}",
    "-ffp-contract=off", "-fno-slp-vectorize", "-fvisibility=hidden", "-Wall", "-Wno-unused-function",
    "-Wno-unused-variable", "-Wno-unused-but-set-variable",
    f"-I{INCLUDE}", f"-I{CSRC}",
]


def _sources() -> list[Path]:
    return sorted([*CSRC.glob("*.hip"), *CSRC.glob("*.cpp")])


def _headers_mtime() -> float:
    hs = [*CSRC.glob("*.h"), *INCLUDE.glob("*.h")]
    return max((h.stat().st_mtime for h in hs), default=0.0)


# Per-source extra flags (none). Tried: `-mllvm -amdgpu-mfma-vgpr-form` on match_hamming.hip (MFMA
# accumulators in VGPRs, no accvgpr copies) returned wrong Hamming distances for a few pairs with two
# MFMA row tiles per staged train tile (deterministic per grid shape, gone without the flag): not used.
EXTRA: dict = {}


def _compile(src: Path, hmt: float) -> Path:
    obj = BUILD / (src.name + ".o")
    if obj.exists() and obj.stat().st_mtime > max(src.stat().st_mtime, hmt, Path(__file__).stat().st_mtime):
        return obj
    cmd = [HIPCC, *CFLAGS, *EXTRA.get(src.name, []), "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed on {src.name}:\n{r.stderr}")
    return obj


def build(verbose: bool = False) -> Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    LIBDIR.mkdir(parents=True, exist_ok=True)
    hmt = _headers_mtime()
    srcs = _sources()
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        objs = list(ex.map(lambda s: _compile(s, hmt), srcs))
    newest = max(o.stat().st_mtime for o in objs)
    if not LIB.exists() or LIB.stat().st_mtime < newest:
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(LIB), *map(str, objs)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
