"""Host-code sanitizers: the oracle's C sources and the host-compiled copy of the
per-hypothesis kernel code (minicv_amd/csrc/hyp_*.h) built with AddressSanitizer + UBSan and run
by tests/native/san_driver.cpp, which also checks the two against each other bit for bit.
GPU ASan / xnack+ code objects are not available on this pool, so the device side is covered by
the bit-exact GPU parity tests instead. CPU only."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1",
       "-ffp-contract=off", "-fno-fast-math", "-mfma", "-fopenmp"]


@pytest.mark.skipif(shutil.which("gcc") is None or shutil.which("g++") is None, reason="needs gcc / g++")
def test_host_code_under_asan_ubsan(tmp_path):
    objs = []
    for c in ("oracle.c", "oracle_e.c", "oracle_pnp.c", "oracle_epnp.c", "oracle_f7.c", "oracle_scaled.c", "oracle_sqpnp.c"):
        o = tmp_path / (c + ".o")
        subprocess.run(["gcc", "-std=c11", *SAN, "-c", str(ROOT / "oracle" / c), "-o", str(o)], check=True,
                       capture_output=True, text=True)
        objs.append(str(o))
    exe = tmp_path / "san_driver"
    r = subprocess.run(["g++", "-std=c++17", *SAN, f"-I{ROOT / 'minicv_amd' / 'csrc'}", f"-I{ROOT / 'include'}",
                        str(ROOT / "tests" / "native" / "san_driver.cpp"), *objs, "-o", str(exe), "-lm"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    run = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600,
                         env={"ASAN_OPTIONS": "detect_leaks=1", "UBSAN_OPTIONS": "print_stacktrace=1",
                              "OMP_NUM_THREADS": "2"})
    assert run.returncode == 0, (run.stdout + run.stderr)[-4000:]
    assert run.stdout.startswith("san ok"), run.stdout
