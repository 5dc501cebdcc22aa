#!/usr/bin/env python3
"""Copy the judged evidence from gpurun_out/ (scratch) into profiles/ (tracked):
  gpurun_out/bench_<w>.log           -> profiles/<round>_bench_<w>.json   (the bench JSON line)
  gpurun_out/prof_<w>/run_kernel_stats.csv -> profiles/<round>/kernel_stats_<w>.csv
  gpurun_out/pmc_{fetch,write}_<w>/run_counter_collection.csv -> profiles/<round>/pmc_{fetch,write}_<w>.csv
  gpurun_out/pmc_sq_<w>/run_counter_collection.csv -> profiles/<round>/pmc_sq_<w>.csv
and derive profiles/pmc_traffic.json: HBM bytes per launch of each workload's dominant kernel
(FETCH_SIZE x2 + WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md), keyed by kernel with
the workload config it was measured on (bench.py reads it for `roofline.traffic`), plus each sweep's
SQ counters and the VALU instructions per evaluation derived from them (bench.py's `roofline.issue`). Usage: collect_profiles.py r01
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
WORKLOADS = ["homography", "fundamental", "essential", "pnp", "hamming", "l2", "scaled"]
# dominant kernel per BASELINE workload (substring of the demangled rocprofv3 kernel name)
KERNELS = {"homography": "mcv_h_verify_cert", "fundamental": "mcv_f_verify", "hamming": "mcv_hamming_mfma",
           "l2": "mcv_l2_gemm", "essential": "mcv_e_verify", "pnp": "mcv_pnp_verify",
           "scaled": "mcv_scaled_costs"}
EXTRA_BENCH = ["homography_fused", "homography_fast", "pnp_ap3p", "essential_fast"]   # second bench lines (bench_<name>.log)


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
    for w in WORKLOADS + EXTRA_BENCH:
        log = OUT / f"bench_{w}.log"
        if log.exists() and (j := last_json(log)):
            (PROF / f"{rnd}_bench_{w}.json").write_text(json.dumps(j) + "\n")
            print("bench", w, j["value"])
        ks = OUT / f"prof_{w}" / "run_kernel_stats.csv"
        if ks.exists():
            shutil.copy(ks, PROF / rnd / f"kernel_stats_{w}.csv")
    traffic = {}
    mean = lambda xs: sum(xs) / len(xs)
    median = lambda xs: sorted(xs)[len(xs) // 2] if len(xs) % 2 else sum(sorted(xs)[len(xs) // 2 - 1:len(xs) // 2 + 1]) / 2
    for w, kernel in KERNELS.items():
        j = last_json(PROF / f"{rnd}_bench_{w}.json") if (PROF / f"{rnd}_bench_{w}.json").exists() else None
        if not j:
            continue
        c = j["config"]
        if w == "homography":
            config, alg = f"{c.get('correspondences')}x{c.get('hypotheses_per_gpu')}", \
                16.0 * c.get("correspondences", 0) * c.get("hypotheses_per_gpu", 0)
        elif w == "fundamental":
            config, alg = f"{c.get('correspondences')}x{c.get('hypotheses_total')}", \
                16.0 * c.get("correspondences", 0) * c.get("hypotheses_total", 0)
        elif w == "essential":
            models = j.get("roofline", {}).get("models_per_launch", 0)
            config, alg = f"{c.get('correspondences')}x{c.get('hypotheses_total')}", \
                16.0 * c.get("correspondences", 0) * models
        elif w == "pnp":
            config, alg = f"{c.get('correspondences')}x{c.get('hypotheses_total')}", \
                20.0 * c.get("correspondences", 0) * c.get("hypotheses_total", 0)
        elif w == "scaled":   # 2 N candidates x N observations x 40 B (world point + observation)
            config, alg = f"{c.get('observations')}", 80.0 * c.get("observations", 0) ** 2
        else:
            config = f"{c.get('queries')}x{c.get('train')}"
            dim_bytes = 32.0 if w == "hamming" else 512.0
            alg = dim_bytes * c.get("queries", 0) * c.get("train", 0)
        t = {"workload": w, "config": config, "algorithmic_bytes_per_launch": alg,
             "source": f"rocprofv3 --kernel-trace --pmc (one counter per pass), bench.py, round {rnd}"}
        fetch = OUT / f"pmc_fetch_{w}" / "run_counter_collection.csv"
        write = OUT / f"pmc_write_{w}" / "run_counter_collection.csv"
        if fetch.exists() and write.exists():
            shutil.copy(fetch, PROF / rnd / f"pmc_fetch_{w}.csv")
            shutil.copy(write, PROF / rnd / f"pmc_write_{w}.csv")
            f = pmc_sums(fetch, kernel).get("FETCH_SIZE")
            wr = pmc_sums(write, kernel).get("WRITE_SIZE")
            if f and wr:
                # the median dispatch: a dispatch's counts also take the write-backs of lines the kernels
                # before it left dirty (round 6: one E dispatch of five wrote 168 MiB against 41.1-41.2)
                t.update({"FETCH_SIZE_KB": median(f), "WRITE_SIZE_KB": median(wr), "dispatches": len(f),
                          "WRITE_SIZE_KB_range": [min(wr), max(wr)], "statistic": "median over the dispatches",
                          "hbm_bytes_per_launch": (2 * median(f) + median(wr)) * 1024.0})
                print("traffic", kernel, t["hbm_bytes_per_launch"])
        # MFMA SQ pass (matchers): MFMA instructions, MFMA busy share of the SIMD cycles
        mf_src = OUT / f"pmc_mfma_{w}" / "run_counter_collection.csv"
        if mf_src.exists():
            shutil.copy(mf_src, PROF / rnd / f"pmc_mfma_{w}.csv")
            sq = {k: mean(v) for k, v in sorted(pmc_sums(mf_src, kernel).items())}
            d = {"sq": sq}
            if sq.get("GRBM_GUI_ACTIVE") and sq.get("SQ_VALU_MFMA_BUSY_CYCLES"):
                cyc = sq["GRBM_GUI_ACTIVE"] / 8
                # SQ_VALU_MFMA_BUSY_CYCLES counts cycles (MI355X_MICROARCH.md), summed over the 1024 SIMDs
                d["derived"] = {"kernel_cycles": cyc, "mfma_busy": sq["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc)}
                print("mfma", kernel, d["derived"])
            t["counters"] = d
        # SQ pass (SQ_INSTS_VALU & co.): measured VALU instructions per evaluation and VALU busy share
        sq_src = OUT / f"pmc_sq_{w}" / "run_counter_collection.csv"
        if not sq_src.exists() and w == "homography":
            sq_src = OUT / "pmc_sq" / "run_counter_collection.csv"
        if sq_src.exists():
            shutil.copy(sq_src, PROF / rnd / f"pmc_sq_{w}.csv")
            sq = {k: mean(v) for k, v in sorted(pmc_sums(sq_src, kernel).items())}
            d = {"sq": sq}
            ms = j.get("roofline", {}).get("avg_launch_ms")
            if sq.get("GRBM_GUI_ACTIVE") and sq.get("SQ_INSTS_VALU") and ms:
                evals = alg / (20.0 if w == "pnp" else 16.0)
                cyc = sq["GRBM_GUI_ACTIVE"] / 8          # summed over the 8 XCDs' GRBM instances
                d["derived"] = {"clock_GHz": cyc / (ms * 1e-3) / 1e9,
                                "valu_instr_per_eval": sq["SQ_INSTS_VALU"] * 64 / evals,
                                # one wave64 VALU instruction occupies a SIMD for 4 cycles; 1024 SIMDs
                                "valu_busy": sq["SQ_INSTS_VALU"] * 4 / (1024 * cyc)}
                print("sq", kernel, d["derived"])
            t["counters"] = d
        if "hbm_bytes_per_launch" in t or "counters" in t:
            traffic[kernel] = t
    lds = OUT / "pmc_lds_homography" / "run_counter_collection.csv"
    if lds.exists():
        shutil.copy(lds, PROF / rnd / "pmc_lds_homography.csv")
    # extra screens: raw SQ counters of named kernels (e.g. the H generate, lane vs quad form)
    for src in sorted(OUT.glob("pmc_gen_*")):
        f = src / "run_counter_collection.csv"
        if f.exists():
            shutil.copy(f, PROF / rnd / f"{src.name}.csv")
    if traffic:
        # merge: entries not re-measured this round stay as they were (their config says what they measured)
        old = PROF / "pmc_traffic.json"
        merged = json.loads(old.read_text()) if old.exists() else {}
        merged.update(traffic)
        traffic = merged
        for v in traffic.values():
            v.setdefault("correction", "FETCH_SIZE x2 (gfx950 counts half of a wide streaming read, MI355X_MICROARCH.md "
                                       "HBM) + WRITE_SIZE; units KB")
        (PROF / "pmc_traffic.json").write_text(json.dumps(traffic, indent=1) + "\n")


if __name__ == "__main__":
    main()
