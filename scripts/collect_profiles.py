#!/usr/bin/env python3
"""Copy the judged evidence from gpurun_out/ (scratch) into profiles/ (tracked):
  gpurun_out/bench_<w>.log           -> profiles/<round>_bench_<w>.json   (the bench JSON line)
  gpurun_out/prof_<w>/run_kernel_stats.csv -> profiles/<round>/kernel_stats_<w>.csv
  gpurun_out/pmc_{fetch,write,sq}/run_counter_collection.csv -> profiles/<round>/pmc_*_counters.csv
and derive profiles/pmc_h_verify.json (HBM bytes per mcv_h_verify launch with the gfx950
FETCH_SIZE x2 correction of MI355X_MICROARCH.md, plus SQ counters). Usage: collect_profiles.py r01
"""
import csv
import json
import shutil
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
OUT = ROOT / "gpurun_out"
PROF = ROOT / "profiles"
WORKLOADS = ["homography", "fundamental", "essential", "pnp", "hamming", "l2"]


def last_json(path: Path):
    for line in reversed(path.read_text().splitlines()):
        line = line.strip()
        if line.startswith("{"):
            return json.loads(line)
    return None


def pmc_sums(path: Path, kernel_prefix: str):
    """counter -> list of per-dispatch values for kernels whose name contains kernel_prefix."""
    per = defaultdict(lambda: defaultdict(float))
    with path.open() as f:
        for row in csv.DictReader(f):
            if kernel_prefix in row["Kernel_Name"]:
                per[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
    out = defaultdict(list)
    for d in per.values():
        for k, v in d.items():
            out[k].append(v)
    return out


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
    (PROF / rnd).mkdir(parents=True, exist_ok=True)
    for w in WORKLOADS:
        log = OUT / f"bench_{w}.log"
        if log.exists() and (j := last_json(log)):
            (PROF / f"{rnd}_bench_{w}.json").write_text(json.dumps(j) + "\n")
            print("bench", w, j["value"])
        ks = OUT / f"prof_{w}" / "run_kernel_stats.csv"
        if ks.exists():
            shutil.copy(ks, PROF / rnd / f"kernel_stats_{w}.csv")
    pmc = {}
    for name in ("fetch", "write", "sq"):
        src = OUT / f"pmc_{name}" / "run_counter_collection.csv"
        if src.exists():
            shutil.copy(src, PROF / rnd / f"pmc_{name}_counters.csv")
            pmc[name] = pmc_sums(src, "mcv_h_verify")
    if {"fetch", "write"} <= pmc.keys() and pmc["fetch"].get("FETCH_SIZE"):
        hb = json.loads((PROF / f"{rnd}_bench_homography.json").read_text())
        n = hb["config"]["correspondences"]
        hyps = hb["config"]["hypotheses_per_gpu"]
        mean = lambda xs: sum(xs) / len(xs)
        fetch_kb = mean(pmc["fetch"]["FETCH_SIZE"])
        write_kb = mean(pmc["write"]["WRITE_SIZE"])
        sq = {k: mean(v) for k, v in sorted(pmc.get("sq", {}).items())}
        d = {
            "kernel": "mcv_h_verify (default variant)", "n": n, "hyps": hyps,
            "FETCH_SIZE_KB": fetch_kb, "WRITE_SIZE_KB": write_kb,
            "hbm_bytes_per_launch": (2 * fetch_kb + write_kb) * 1024.0,
            "correction": "FETCH_SIZE x2 (gfx950 counts half of a wide streaming read, MI355X_MICROARCH.md HBM); "
                          "WRITE_SIZE as reported; units KB",
            "algorithmic_bytes_per_launch": 16 * n * hyps,
            "sq": sq,
            "source": f"rocprofv3 --kernel-trace --pmc (three separate passes), bench.py --steps 3, round {rnd}",
        }
        if sq.get("GRBM_GUI_ACTIVE") and sq.get("SQ_INSTS_VALU"):
            ms = hb["roofline"]["avg_launch_ms"]
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs' GRBM instances
            d["derived"] = {"clock_GHz": sq["GRBM_GUI_ACTIVE"] / 8 / (ms * 1e-3) / 1e9,
                            "valu_instr_per_eval": sq["SQ_INSTS_VALU"] * 64 / (n * hyps)}
        (PROF / "pmc_h_verify.json").write_text(json.dumps(d, indent=1) + "\n")
        print("pmc", d["hbm_bytes_per_launch"], d.get("derived"))


if __name__ == "__main__":
    main()
