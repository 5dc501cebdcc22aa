#!/usr/bin/env python3
"""Headline benchmark: RANSAC hypotheses/sec at 100k correspondences (BASELINE.json `metric`,
config[2]: findHomography RANSAC, 100k correspondences x 1M hypotheses, 1 MI355X).

A step = one findHomography RANSAC call on HBM-resident correspondences (packed float4, seeded
synthetic data of the cfg3 shape): generate + minimal-solve + inlier-count 1M hypotheses
(per GPU), reduce to the best packed key (RCCL all-reduce MAX across ranks when N > 1), then
finalize: mask of the winner, refit on its inliers and 10 LM iterations.

Scaling: weak — each GPU evaluates its own 1M-hypothesis batch of the same problem (the union is
one RANSAC call over N x 1M hypotheses), one 16-byte all-reduce per step.

Printed JSON carries the live roofline of the dominant kernel (mcv_h_verify_pk, HIP events on its
launch stream; algorithmic bytes = 16 B x N correspondences per hypothesis) and the oracle's CPU
throughput on a bounded sample of the same workload (rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

N_CORR = 100_000
HYPS_PER_GPU = 1 << 20
F_N_CORR = 500_000            # BASELINE config[3]: findFundamentalMat 8-pt, 500k correspondences
F_HYPS_TOTAL = 1 << 20        # hypotheses per call, sharded over the ranks (strong scaling; SURVEY.md:125,410)
F_SEED = 4
E_N_CORR = 100_000            # essential (cvRecoverPose path): not a BASELINE config
E_HYPS_TOTAL = 1 << 20        # as cfg4: 131072 hypotheses per rank at 8 ranks
E_SEED = 6
E_FOCAL, E_PP, E_THR_PX = 800.0, (640.0, 360.0), 1.0
P_N_CORR = 20_000             # PnP (cvSolvePnPRansac path): reference testPnp size (Program.fs:14)
P_HYPS_TOTAL = 1 << 20
P_FLOPS_PER_EVAL = 51         # pnp_project: R X + t (18), 1 / Zc (1), distortion + intrinsics (32)
P_SEED = 8
P_THR_PX = 2.0
THR = 5e-3
SEED = 3
HBM_PEAK_GBPS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# Roofs (MI355X_MICROARCH.md): fp32 vector = fp32-input MFMA = 157.3 TFLOP/s dense, fp64 vector 78.6;
# the int32 VALU op rate is the fp32 FMA lane rate counted once per op (256 CUs x 4 SIMDs x 32 lanes
# x 2.4 GHz).
FP32_PEAK_TF = 157.3
FP64_PEAK_TF = 78.6
# The reference's projectPoints / avgReprojectionError arithmetic is op-by-op fp64 (no contraction:
# OpenCV's x86-64 build, the managed F# code): every add and mul is its own instruction, so the
# attainable flop rate of that arithmetic is half the FMA-counted fp64 peak.
FP64_NOFMA_PEAK_TF = FP64_PEAK_TF / 2
FP32_MFMA_PEAK_TF = 157.3
F16_MFMA_PEAK_TF = 2516.6      # dense f16 MFMA: 32x32x16 = 16384 MAC per 32 cycles per SIMD, 1024 SIMDs, 2.4 GHz
INT32_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
I8_MFMA_PEAK_TOPS = 2 * F16_MFMA_PEAK_TF   # MI355X_MICROARCH.md: i8 32x32x32 at the cycles of bf16 32x32x16
FP4_MFMA_PEAK_TOPS = 4 * F16_MFMA_PEAK_TF  # MI355X_MICROARCH.md: fp4 32x32x64 at the cycles of bf16 32x32x16
# Algorithmic work per unit: homography computeError = 25 flops per (hypothesis,
# correspondence) (3 dot products, 1 reciprocal, 2 sub, 2 mul, 1 add, 1 compare); Sampson error =
# 34 fp64 flops per (model, correspondence) (F x1 12, F^T x2 8, x2^T F x1 4, denominator 7, c^2,
# division, compare); Hamming = 24 int32 ops per (query, train) pair of 256-bit descriptors
# (8 xor + 8 popcount + 7 add + 1 compare).
H_FLOPS_PER_EVAL = 25
SAMPSON_FLOPS_PER_EVAL = 34
HAM_OPS_PER_PAIR = 24
MATCHER_PROF_STRIDE = 5       # matchers: HIP events around every 5th GEMM launch of the timed loop
# Issue models (secondary: what the kernels' instruction streams allow at 2.4 GHz, SIMD cycles per
# 64 evaluations; measured issue costs: VOP3/VOP3P 4 cycles, VOP2/VOPC e32 2, transcendental 8):
#   Sampson prefilter (F, E): 56 per (model, correspondence); Hamming 58 per pair. The homography
#   sweeps use the measured VALU instruction count instead (measured_issue, from the SQ pass).
SPK_CYC_PER_WAVE_EVAL = 56
# Certified PnP prefilter (pnp_pk.h): per point pair (two lanes' worth of evaluations) 40 packed
# ops at 4 cycles, 2 v_rcp_f32 at 8, 2 v_max_f32 + 2 v_mul_f32 + 6 v_cmp (VOP3) at 4 = 216 cycles
# per 128 (pose, point) evaluations.
PPK_CYC_PER_WAVE_EVAL = 108
HAMMING_CYC_PER_WAVE_PAIR = 58
SIMD_CYC_PER_S = 256 * 4 * 2.4e9


def issue_peak(cycles_per_64: float) -> float:
    """Evaluations / s when every SIMD issues the kernel's stream back to back (64 lanes per wave)."""
    return SIMD_CYC_PER_S / cycles_per_64 * 64


def host_cpu():
    """The host the CPU baseline runs on: threads used (OMP_NUM_THREADS, which the GPU box sets to
    its CPU share, else every core this process may run on), nproc and the CPU model."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return {"threads": env or aff, "nproc": os.cpu_count(), "affinity": aff, "model": model,
            "threads_from": "OMP_NUM_THREADS" if env else "sched_getaffinity"}


def cpu_threads() -> int:
    return host_cpu()["threads"]


def dist_setup(torch, dist):
    """(world, rank, device) for this process. The driver runs N ranks on N GPUs over RCCL
    ("nccl"); MCV_DIST_BACKEND=gloo rehearses N ranks on the GPUs this box has (ranks share a
    device, the one all-reduce goes through gloo) — a test of the multi-rank path, not a benchmark."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("MCV_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend != "nccl":
        local = local % max(ndev, 1)
    elif local >= ndev:
        raise SystemExit(f"rank {rank}: {world} ranks over RCCL need {world} visible GPUs, this box has {ndev} "
                         "(MCV_DIST_BACKEND=gloo rehearses the ranks on a shared device)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    return world, rank, dev

def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--hyps", type=int, default=HYPS_PER_GPU, help="hypotheses per GPU per step")
    ap.add_argument("--n", type=int, default=N_CORR)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--hamming-form", default="gemm", choices=["gemm", "popcount"],
                    help="Hamming kernel: fp4 GEMM on the matrix cores (default) or the XOR / popcount sweep")
    ap.add_argument("--pnp-kind", default="EPNP", choices=["Iterative", "EPNP", "P3P", "DLS", "UPNP", "AP3P"],
                    help="pnp workload: the reference's solverKind (EPNP = its own testPnp, Program.fs:27-32)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary fast_minimal leg of the H / F lines (profiling runs: one solver per process)")
    ap.add_argument("--fast-minimal", action="store_true",
                    help="opt-in elimination minimal solver for H / 8-point F (default: OpenCV's cv::eigen runKernel)")
    ap.add_argument("--fused", action="store_true",
                    help="opt-in FMA-contracted inlier error (default: OpenCV's op-by-op order, the reference's)")
    ap.add_argument("--workload", default="homography",
                    choices=["homography", "fundamental", "essential", "pnp", "hamming", "l2", "scaled"],
                    help="homography = the headline (BASELINE config[2]); the others are config[1], [3], [4]")
    return ap.parse_args()


def cpu_baseline(src, dst, target_s: float):
    """Oracle (plain-C restatement, OpenMP over hypotheses) on a bounded sample of the same workload."""
    sys.path.insert(0, str(ROOT / "tests"))
    import numpy as np
    import _oracle as O
    pts4 = O.pack4(src, dst)
    thr2 = float(np.float32(THR * THR))
    threads = cpu_threads()
    t = time.perf_counter()
    O.h_counts(pts4, SEED, 0, 4 * threads, thr2, threads)
    cal = (time.perf_counter() - t) / (4 * threads)
    sample = max(4 * threads, int(target_s / max(cal, 1e-6)))
    t = time.perf_counter()
    O.h_counts(pts4, SEED, 0, sample, thr2, threads)
    el = time.perf_counter() - t
    return {"value": sample / el, "unit": "hypotheses/s", "cores": threads, "kind": "port", "host": host_cpu(),
            "sample": f"{sample} hypotheses x {src.shape[0]} correspondences (sample+solve+fp32 op-by-op count), "
                      f"oracle/oracle.c, OpenMP {threads} threads, {el:.1f} s"}


def cpu_baseline_f(a, b, target_s: float):
    sys.path.insert(0, str(ROOT / "tests"))
    import numpy as np
    import _oracle as O
    pts4 = O.pack4(a, b)
    thr2 = float(np.float32(THR * THR))
    threads = cpu_threads()
    t = time.perf_counter()
    O.f_counts(pts4, F_SEED, 0, 2 * threads, thr2, 1, threads)
    cal = (time.perf_counter() - t) / (2 * threads)
    sample = max(2 * threads, int(target_s / max(cal, 1e-6)))
    t = time.perf_counter()
    O.f_counts(pts4, F_SEED, 0, sample, thr2, 1, threads)
    el = time.perf_counter() - t
    return {"value": sample / el, "unit": "hypotheses/s", "cores": threads, "kind": "port", "host": host_cpu(),
            "sample": f"{sample} hypotheses x {a.shape[0]} correspondences (8-pt sample+solve+fp64 Sampson "
                      f"count), oracle/oracle.c, OpenMP {threads} threads, {el:.1f} s"}


def bench_matcher(args):
    """BASELINE config[1] (Hamming 10k x 10k x 256 bit) / config[4] (L2 SIFT-128 50k x 50k, fp32 MFMA).
    Queries are sharded over ranks (no collective); the train set is replicated."""
    import numpy as np
    import torch
    import torch.distributed as dist
    world, rank, dev = dist_setup(torch, dist)
    from minicv_amd import native as NL, synthetic as S, device as D
    from minicv_amd import dist as MD
    ham = args.workload == "hamming"
    if ham:
        nq, nt = 10_000, 10_000
        q, t, _ = S.hamming_problem(nq, nt, seed=2)
        qd, td = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
    else:
        nq, nt = 50_000, 50_000
        q, t, _ = S.l2_problem(nq, nt, dim=128, seed=5)
        qd, td = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
    b0, cnt = MD.shard(nq, rank, world)
    qs = qd[b0:b0 + cnt].contiguous()
    idx = torch.empty(cnt, dtype=torch.int32, device=dev)
    idx2 = torch.empty_like(idx)
    dist_t = torch.empty(cnt, dtype=torch.int32 if ham else torch.float32, device=dev)
    dist2 = torch.empty_like(dist_t)

    def step():
        if ham:
            D.match_hamming(qs, td, idx, dist_t, idx2, dist2, form=args.hamming_form)
        else:
            D.match_l2(qs, td, idx, dist_t, idx2, dist2)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    NL.lib().mcvProfileReset()
    # every MATCHER_PROF_STRIDE-th GEMM launch is timed: an event pair costs the stream ~3 us each way,
    # which a 36 us Hamming step would otherwise carry on every step (scripts/exp/ham_gap.py)
    NL.lib().mcvProfileEnable(MATCHER_PROF_STRIDE)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    NL.lib().mcvProfileEnable(0)
    import ctypes as C
    kms = C.c_double(0)
    launches = NL.lib().mcvProfileRead(b"hamming" if ham else b"l2_mfma", C.addressof(kms))
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    if rank == 0:
        avg_ms = kms.value / max(launches, 1)
        if ham:
            pairs = cnt * nt
            ach = pairs / (avg_ms * 1e-3)
            gemm = args.hamming_form == "gemm"
            kp = 256   # 32-byte descriptors: 256 fp4 elements per expanded row
            mfma_roof = {"bound": "mfma-fp4", "achieved": 2.0 * kp * ach / 1e12, "peak": FP4_MFMA_PEAK_TOPS,
                         "unit": "Tops/s", "frac": 2.0 * kp * ach / 1e12 / FP4_MFMA_PEAK_TOPS,
                         "traffic": load_traffic("mcv_hamming_mfma", f"{nq}x{nt}"), "kernel": "mcv_hamming_mfma",
                         "avg_launch_ms": avg_ms, "timed_launches": launches,
                         "timed_every": MATCHER_PROF_STRIDE,
                         "model": "Hamming as an fp4 GEMM: [nt x 256] x [256 x nq] on v_mfma_f32_32x32x64_f8f6f4 "
                                  "(2 x 256 fp4 ops per pair; products t (1 - 2 q), sum = ham - popcount(q)), exact "
                                  f"in f32; against the i8 form's peak: {2.0 * kp * ach / 1e12 / I8_MFMA_PEAK_TOPS:.3f}; "
                                  f"the popcount view: {HAM_OPS_PER_PAIR * ach / 1e12:.1f} of {INT32_PEAK_TOPS:.1f} "
                                  "int32 Tops/s at 24 ops per pair"}
            line = {"metric": "BF Hamming knn-2 queries/sec, 10k x 10k 256-bit (BASELINE config[1])",
                    "value": nq * args.steps / el, "unit": "queries/s",
                    "hamming_form": "fp4 GEMM on the matrix cores (default)" if gemm else
                                    "XOR / popcount sweep (--hamming-form popcount)",
                    "roofline": mfma_roof if gemm else {"bound": "int-valu", "achieved": HAM_OPS_PER_PAIR * ach / 1e12,
                                 "peak": INT32_PEAK_TOPS, "unit": "Tops/s",
                                 "frac": HAM_OPS_PER_PAIR * ach / 1e12 / INT32_PEAK_TOPS,
                                 "traffic": load_traffic("mcv_hamming_partial", f"{nq}x{nt}"),
                                 "kernel": "mcv_hamming_partial", "avg_launch_ms": avg_ms,
                                 "model": f"{HAM_OPS_PER_PAIR} int32 ops per (query, train) pair of 256-bit "
                                          "descriptors",
                                 "hbm": {"effective_GBps": 32.0 * pairs / (avg_ms * 1e-3) / 1e9,
                                         "peak": HBM_PEAK_GBPS,
                                         "note": "32 B x Nt per query as if streamed; the 640 KB sets are "
                                                 "L2-resident"},
                                 "issue": {"achieved": ach, "peak": issue_peak(HAMMING_CYC_PER_WAVE_PAIR),
                                           "unit": "pairs/s", "frac": ach / issue_peak(HAMMING_CYC_PER_WAVE_PAIR),
                                           "model": f"{HAMMING_CYC_PER_WAVE_PAIR} SIMD cycles per 64 (query, "
                                                    "train) pairs at 2.4 GHz"}},
                    "dtype": "fp4" if gemm else "u32", "scaling": "strong"}
        else:
            exact_scans = NL.lib().mcvL2LastExactScans()
            form = NL.lib().mcvL2LastGemmForm()
            flops = 2.0 * cnt * nt * 128
            tf = flops / (avg_ms * 1e-3) / 1e12
            if form == 16:   # f16-split GEMM form: three f16 MFMA products per (query, train, dim)
                roof = {"bound": "mfma-f16", "achieved": 3.0 * tf, "peak": F16_MFMA_PEAK_TF, "unit": "TFLOP/s",
                        "frac": 3.0 * tf / F16_MFMA_PEAK_TF,
                        "kernel": "mcv_l2_gemm",
                        "model": "fp32 operands split into f16 hi + lo; hi.hi + hi.lo + lo.hi on "
                                 "v_mfma_f32_32x32x16_f16 = 3 x 2 Nq Nt D MFMA flops per launch; "
                                 f"algorithmic rate {tf:.1f} TFLOP/s (2 Nq Nt D)"}
            else:
                roof = {"bound": "mfma", "achieved": tf, "peak": FP32_MFMA_PEAK_TF, "unit": "TFLOP/s",
                        "frac": tf / FP32_MFMA_PEAK_TF, "kernel": "mcv_l2_gemm"}
            roof.update({"traffic": load_traffic(roof["kernel"], f"{nq}x{nt}"), "avg_launch_ms": avg_ms,
                         "timed_launches": launches, "timed_every": MATCHER_PROF_STRIDE})
            line = {"metric": "BF L2 knn-2 TFLOP/s, SIFT-128 50k x 50k fp32 GEMM on MFMA (BASELINE config[4])",
                    "value": 2.0 * nq * nt * 128 * args.steps / el / 1e12, "unit": "TFLOP/s",
                    "roofline": roof,
                    "gemm_form": {16: "f16 split (hi.hi + hi.lo + lo.hi), exact re-rank",
                                  32: "f32, exact re-rank"}.get(form, str(form)),
                    "exact_rerank": {"queries_to_exact_scan": exact_scans,
                                     "note": "idx / dist are the exact direct-sum answer (fp64, ties -> lowest "
                                             "index); the GEMM form only nominates candidates"},
                    "dtype": "f32", "scaling": "strong"}
        line.update({"n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                     "ms_per_step": el / args.steps * 1e3, "higher_is_better": True, "vs_baseline": None,
                     "data": "synthetic (seeded, planted neighbours)",
                     "config": {"workload": args.workload, "queries": nq, "train": nt,
                                "parallelism": f"query-sharded dp{world}"},
                     "cpu_baseline": None})
        if world == 1 and not args.no_cpu_baseline:
            sys.path.insert(0, str(ROOT / "tests"))
            import _oracle as O
            threads = cpu_threads()
            sq = 2000 if ham else 200
            t1 = time.perf_counter()
            (O.match_hamming if ham else O.match_l2)(q[:sq], t, nthreads=threads)
            ct = time.perf_counter() - t1
            line["cpu_baseline"] = {"value": sq / ct if ham else 2.0 * sq * nt * 128 / ct / 1e12,
                                    "unit": "queries/s" if ham else "TFLOP/s", "cores": threads, "kind": "port",
                                    "host": host_cpu(),
                                    "sample": f"{sq} queries x {nt} train, oracle/oracle.c, OpenMP {threads}"}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def measured_issue(kernel: str, config: str, evals_per_s: float):
    """Issue rate of a sweep from its committed SQ counter pass (profiles/pmc_traffic.json:
    SQ_INSTS_VALU per evaluation): every SIMD issuing one wave64 VALU instruction per 4 cycles at
    2.4 GHz. None when no pass was taken on this workload config."""
    p = ROOT / "profiles" / "pmc_traffic.json"
    try:
        d = json.loads(p.read_text()).get(kernel) if p.exists() else None
        der = d["counters"]["derived"] if d and d.get("config") == config else None
        per = der["valu_instr_per_eval"] if der else None
    except Exception:
        der, per = None, None
    if not per:
        return None
    peak = SIMD_CYC_PER_S * 16 / per
    out = {"achieved": evals_per_s, "peak": peak, "unit": "evaluations/s", "frac": evals_per_s / peak,
           "model": f"{per:.2f} VALU lane-instructions per evaluation (rocprofv3 SQ_INSTS_VALU, profiles/"
                    "pmc_traffic.json), one wave64 VALU instruction per SIMD per 4 cycles at 2.4 GHz"}
    if der.get("valu_busy"):   # the counter pass's own share of SIMD cycles with a VALU instruction issuing
        out["valu_busy_measured"] = der["valu_busy"]
        out["clock_GHz_measured"] = der.get("clock_GHz")
    return out


def load_traffic(kernel: str, config: str):
    """HBM bytes per launch of `kernel` on workload `config` from the committed rocprofv3 PMC
    summary (profiles/pmc_traffic.json, written by scripts/collect_profiles.py), if present."""
    p = ROOT / "profiles" / "pmc_traffic.json"
    if not p.exists():
        return None
    try:
        # keys are kernel-name prefixes as rocprofv3 reports them (mcv_f_verify covers mcv_f_verify_pk<..>)
        for key, d in json.loads(p.read_text()).items():
            if (kernel == key or kernel.startswith(key + "_")) and d.get("config") == config:
                return d.get("hbm_bytes_per_launch")
    except Exception:
        return None
    return None


def launch_ranks(n: int) -> int:
    """`--gpus N` (N > 1) without a launcher: start N rank processes of this same command, one per GPU,
    with the environment torch.distributed.run would give them (RANK, LOCAL_RANK, WORLD_SIZE,
    MASTER_ADDR = 127.0.0.1, a free MASTER_PORT), before this process imports torch or touches a GPU
    (the ranks are children, never an exec). Waits for all of them; when one fails the others are
    terminated and its exit code is returned. Rank 0 prints the one JSON line."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-u", str(Path(__file__).resolve()), *sys.argv[1:]]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env))

    def stop_all():
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=15)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    rc = 0
    try:
        while any(p.poll() is None for p in procs):
            bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if bad:
                rc = bad[0]
                stop_all()
                break
            time.sleep(0.1)
        if rc == 0:
            rc = next((p.returncode for p in procs if p.returncode != 0), 0)
    except KeyboardInterrupt:
        stop_all()
        rc = 130
    return 128 - rc if rc < 0 else rc   # a rank killed by signal s -> 128 + s


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks")
    if args.workload in ("hamming", "l2"):
        return bench_matcher(args)
    if args.workload == "scaled":
        return bench_scaled(args)
    return bench_ransac(args)


def bench_ransac(args):
    import numpy as np
    import torch
    import torch.distributed as dist

    world, rank, dev = dist_setup(torch, dist)

    from minicv_amd import native as NL, opencv, synthetic as S
    from minicv_amd import device as D
    from minicv_amd import dist as MD

    fund = args.workload == "fundamental"
    ess = args.workload == "essential"
    if ess:
        return bench_essential(args, world, rank, dev)
    if args.workload == "pnp":
        return bench_pnp(args, world, rank, dev)
    n, hyps = args.n, args.hyps
    if fund:
        n = args.n if args.n != N_CORR else F_N_CORR
        hyps = args.hyps if args.hyps != HYPS_PER_GPU else F_HYPS_TOTAL // world
        src, dst, _, _ = S.fundamental_problem(n, F_SEED)
    else:
        src, dst, _ = S.homography_problem(n, SEED)
    pts = D.pack_points_tensor(src, dst, dev)
    plan = D.RansacPlan(NL.MODEL_FUNDAMENTAL if fund else NL.MODEL_HOMOGRAPHY, n, hyps)
    total = hyps * world
    cfg = opencv.RansacParams(threshold=THR, confidence=0.995, max_iters=total, seed=F_SEED if fund else SEED,
                              fixed_iters=True, fused_error=args.fused, fast_minimal=args.fast_minimal).to_c()
    key = torch.zeros(2, dtype=torch.int64, device=dev)
    mask = torch.zeros(n, dtype=torch.uint8, device=dev)
    red = torch.zeros(2, dtype=torch.int64, device=dev)

    def evaluate(begin, count):
        plan.evaluate(pts, n, cfg, begin, count, key)
        k = key.cpu()   # synchronises the stream
        return int(k[0]), int(k[1])

    def allreduce_max(vals):
        if world == 1:
            return vals
        red.copy_(torch.tensor(vals, dtype=torch.int64))
        dist.all_reduce(red, op=dist.ReduceOp.MAX)
        return [int(v) for v in red.cpu()]

    result = {}

    def step():
        cnt, idx, _ = MD.global_best(evaluate, total, rank, world, allreduce_max)
        if idx < 0:
            raise RuntimeError("no model found")
        fc, H = plan.finalize(pts, n, cfg, idx, mask)
        result.update(count=cnt, idx=idx, final_count=fc, H=H)

    for _ in range(args.warmup):
        step()
    NL.lib().mcvProfileReset()
    NL.lib().mcvProfileEnable(1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    NL.lib().mcvProfileEnable(0)
    import ctypes as C
    kms = C.c_double(0)
    launches = NL.lib().mcvProfileRead(b"f_verify" if fund else b"h_verify", C.addressof(kms))
    gms = C.c_double(0)
    glaunches = NL.lib().mcvProfileRead(b"f_generate" if fund else b"h_generate", C.addressof(gms))
    minimal = {"solver": "elimination, h22 / f22 = 1 (opt-in MCV_FLAG_FAST_MINIMAL)" if args.fast_minimal else
               "OpenCV runKernel / run8Point: 9x9 cv::eigen (JacobiImpl_) (default)",
               "generate_avg_ms": gms.value / max(glaunches, 1)}
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    if rank == 0:
        value = total * args.steps / el
        avg_ms = kms.value / max(launches, 1)
        alg_bytes = 16.0 * n * hyps            # per launch: every hypothesis reads all N float4 pairs
        achieved = alg_bytes / (avg_ms * 1e-3) / 1e9
        hkern = "mcv_h_verify_pk" if args.fused else "mcv_h_verify_cert"
        traffic = load_traffic("mcv_f_verify_pk" if fund else hkern, f"{n}x{hyps}")
        evals_per_s = n * hyps / (avg_ms * 1e-3)
        if not fund:
            tf = H_FLOPS_PER_EVAL * evals_per_s / 1e12
            line = {
                "metric": "RANSAC hypotheses/sec @100k corrs; achieved HBM GB/s vs roofline, 1/2/4/8 GPU",
                "value": value,
                "unit": "hypotheses/s",
                "n_gpus": world,
                "steps": args.steps,
                "warmup": args.warmup,
                "ms_per_step": el / args.steps * 1e3,
                "higher_is_better": True,
                "scaling": "weak",
                "vs_baseline": None,
                "dtype": "f32",
                "data": "synthetic (seeded cfg3 homography problem: cvTest H, 50% outliers, sigma 1e-3)",
                "config": {"workload": f"findHomography RANSAC, {n} correspondences x {hyps} hypotheses per GPU "
                                       f"(fixed iterations) + refit/LM, best model via RCCL all-reduce",
                           "correspondences": n, "hypotheses_per_gpu": hyps, "threshold": THR,
                           "error": "fused (opt-in)" if args.fused else "OpenCV op-by-op (default)",
                           "minimal_solver": minimal["solver"],
                           "parallelism": f"hypothesis-sharded dp{world}"},
                "kernels": {"generate": minimal["generate_avg_ms"], "verify": avg_ms},
                "roofline": {"bound": "fp32-valu", "achieved": tf, "peak": FP32_PEAK_TF, "unit": "TFLOP/s",
                             "frac": tf / FP32_PEAK_TF, "traffic": traffic,
                             "kernel": hkern, "avg_launch_ms": avg_ms, "launches": launches,
                             "flops_per_launch": H_FLOPS_PER_EVAL * n * hyps,
                             "model": f"{H_FLOPS_PER_EVAL} flops per (hypothesis, correspondence) x {n} x {hyps} per "
                                      "launch (SURVEY.md 8d)",
                             "hbm": {"effective_GBps": alg_bytes / (avg_ms * 1e-3) / 1e9,
                                     "algorithmic_bytes_per_launch": alg_bytes, "peak": HBM_PEAK_GBPS,
                                     "note": "16 B x N per hypothesis as if streamed from HBM; the 1.6 MB point "
                                             "set is L2-resident, measured HBM bytes per launch are `traffic`"},
                             "issue": measured_issue(hkern, f"{n}x{hyps}", evals_per_s)},
                "result": {"best_count": result["count"], "best_hyp": result["idx"],
                           "refined_count": result["final_count"]},
            }
        else:
            tf = SAMPSON_FLOPS_PER_EVAL * evals_per_s / 1e12
            line = {
                "metric": "RANSAC hypotheses/sec, findFundamentalMat 8-pt @500k corrs (BASELINE config[3])",
                "value": value,
                "unit": "hypotheses/s",
                "n_gpus": world,
                "steps": args.steps,
                "warmup": args.warmup,
                "ms_per_step": el / args.steps * 1e3,
                "higher_is_better": True,
                "scaling": "strong",
                "vs_baseline": None,
                "dtype": "f64",
                "data": "synthetic (seeded two-view problem, 50% outliers, sigma 1e-3)",
                "config": {"workload": f"findFundamentalMat 8-point RANSAC, {n} correspondences x {total} "
                                       f"hypotheses per call sharded over {world} GPU(s), fp64 Sampson error",
                           "correspondences": n, "hypotheses_total": total, "threshold": THR,
                           "minimal_solver": minimal["solver"],
                           "parallelism": f"hypothesis-sharded dp{world}"},
                "kernels": {"generate": minimal["generate_avg_ms"], "verify": avg_ms},
                "roofline": {"bound": "fp32-valu", "achieved": tf, "peak": FP32_PEAK_TF, "unit": "TFLOP/s",
                             "frac": tf / FP32_PEAK_TF, "traffic": traffic,
                             "kernel": "mcv_f_verify_pk", "avg_launch_ms": avg_ms, "launches": launches,
                             "model": f"{SAMPSON_FLOPS_PER_EVAL} (fp64-definition) flops per (model, correspondence); "
                                      "the sweep decides them with a certified packed-fp32 prefilter, so the fp32 "
                                      "vector roof binds",
                             "hbm": {"effective_GBps": alg_bytes / (avg_ms * 1e-3) / 1e9,
                                     "algorithmic_bytes_per_launch": alg_bytes, "peak": HBM_PEAK_GBPS},
                             "issue": measured_issue("mcv_f_verify", f"{n}x{hyps}", evals_per_s) or
                                      {"achieved": evals_per_s, "peak": issue_peak(SPK_CYC_PER_WAVE_EVAL),
                                       "unit": "evaluations/s",
                                       "frac": evals_per_s / issue_peak(SPK_CYC_PER_WAVE_EVAL),
                                       "model": f"certified packed-fp32 Sampson prefilter: {SPK_CYC_PER_WAVE_EVAL} "
                                                "SIMD cycles per 64 (model, correspondence) at 2.4 GHz"}},
                "result": {"best_count": result["count"], "best_hyp": result["idx"]},
            }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = (cpu_baseline_f if fund else cpu_baseline)(src, dst, args.cpu_seconds)
        else:
            line["cpu_baseline"] = None
        if world == 1 and not args.fast_minimal and not args.no_secondary:
            # the same step with the opt-in elimination minimal solver (a secondary figure, not `value`)
            cfg_default = cfg
            cfg = opencv.RansacParams(threshold=THR, confidence=0.995, max_iters=total,
                                      seed=F_SEED if fund else SEED, fixed_iters=True, fused_error=args.fused,
                                      fast_minimal=True).to_c()
            step()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            fe = (time.perf_counter() - t1) / 3
            cfg = cfg_default
            line["fast_minimal"] = {"value": total / fe, "ms_per_step": fe * 1e3,
                                    "note": "opt-in MCV_FLAG_FAST_MINIMAL (elimination minimal solver), 3 steps; "
                                            "`value` above is the default (OpenCV's cv::eigen runKernel / run8Point)"}
        print(json.dumps(line), flush=True)
    plan.close()
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline_e(pts4d, target_s: float):
    sys.path.insert(0, str(ROOT / "tests"))
    import numpy as np
    import _oracle as O
    thr = E_THR_PX / E_FOCAL
    thr2 = float(np.float32(thr * thr))
    threads = cpu_threads()
    t = time.perf_counter()
    O.e_counts(pts4d, E_SEED, 0, 2 * threads, thr2, 1, threads)
    cal = (time.perf_counter() - t) / (2 * threads)
    sample = max(2 * threads, int(target_s / max(cal, 1e-6)))
    t = time.perf_counter()
    O.e_counts(pts4d, E_SEED, 0, sample, thr2, 1, threads)
    el = time.perf_counter() - t
    return {"value": sample / el, "unit": "hypotheses/s", "cores": threads, "kind": "port", "host": host_cpu(),
            "sample": f"{sample} hypotheses x {pts4d.shape[0]} correspondences (5-pt sample+solve, <= 10 models, "
                      f"fp64 Sampson count), oracle/oracle_e.c, OpenMP {threads} threads, {el:.1f} s"}


def bench_essential(args, world, rank, dev):
    """E-RANSAC (the cvRecoverPose path): a step = one findEssentialMat RANSAC call over a fixed
    hypothesis budget on HBM-resident normalised correspondences (hypotheses sharded over ranks,
    one all-reduce), then the winner's mask and the recoverPose cheirality pass."""
    import ctypes as C
    import numpy as np
    import torch
    import torch.distributed as dist
    from minicv_amd import native as NL, opencv, synthetic as S
    from minicv_amd import device as D
    from minicv_amd import dist as MD

    n = args.n if args.n != N_CORR else E_N_CORR
    hyps = args.hyps if args.hyps != HYPS_PER_GPU else E_HYPS_TOTAL // world
    total = hyps * world
    a, b, *_ = S.essential_problem(n, seed=E_SEED, outlier_frac=0.5)
    pts = D.pack_essential_tensor(a, b, E_FOCAL, E_PP, dev)
    plan = D.RansacPlan(NL.MODEL_ESSENTIAL, n, hyps)
    cfg = opencv.RansacParams(threshold=E_THR_PX / E_FOCAL, confidence=0.999, max_iters=total, seed=E_SEED,
                              fixed_iters=True, fused_error=args.fused, fast_minimal=args.fast_minimal).to_c()
    key = torch.zeros(2, dtype=torch.int64, device=dev)
    mask = torch.zeros(n, dtype=torch.uint8, device=dev)
    red = torch.zeros(2, dtype=torch.int64, device=dev)

    def evaluate(begin, count):
        plan.evaluate(pts, n, cfg, begin, count, key)
        k = key.cpu()
        return int(k[0]), int(k[1])

    def allreduce_max(vals):
        if world == 1:
            return vals
        red.copy_(torch.tensor(vals, dtype=torch.int64))
        dist.all_reduce(red, op=dist.ReduceOp.MAX)
        return [int(v) for v in red.cpu()]

    result = {}

    def step():
        cnt, slot, _ = MD.global_best(evaluate, total, rank, world, allreduce_max, slots=NL.E_SLOTS)
        if slot < 0:
            raise RuntimeError("no model found")
        fc, E = plan.finalize(pts, n, cfg, slot, mask)
        result.update(count=cnt, slot=slot, final_count=fc)

    for _ in range(args.warmup):
        step()
    NL.lib().mcvProfileReset()
    NL.lib().mcvProfileEnable(1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    NL.lib().mcvProfileEnable(0)
    vms, gms = C.c_double(0), C.c_double(0)
    vl = NL.lib().mcvProfileRead(b"e_verify", C.addressof(vms))
    gl = NL.lib().mcvProfileRead(b"e_generate", C.addressof(gms))
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    # models per verify launch (the sweep runs over the dense model list): count them once, untimed
    slots = torch.zeros(hyps * NL.E_SLOTS, dtype=torch.int32, device=dev)
    plan.evaluate(pts, n, cfg, rank * hyps, hyps, key, slots)
    models = int((slots >= 0).sum().item())
    if rank == 0:
        v_ms = vms.value / max(vl, 1)
        g_ms = gms.value / max(gl, 1)
        alg_bytes = 16.0 * n * models            # each model reads all N float4 correspondences
        e_tf = SAMPSON_FLOPS_PER_EVAL * n * models / (v_ms * 1e-3) / 1e12
        line = {
            "metric": "RANSAC hypotheses/sec, findEssentialMat 5-pt (cvRecoverPose path) @100k corrs",
            "value": total * args.steps / el, "unit": "hypotheses/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded calibrated two-view problem, 50% outliers, sigma 0.3 px, f 800)",
            "config": {"workload": f"findEssentialMat five-point RANSAC, {n} correspondences x {total} hypotheses "
                                   f"(<= 10 models each) per call sharded over {world} GPU(s)",
                       "correspondences": n, "hypotheses_total": total, "threshold_px": E_THR_PX,
                       "minimal_solver": "Illinois real roots (opt-in MCV_FLAG_FAST_MINIMAL)" if args.fast_minimal
                       else "fivepoint.cpp (getCoeffMat terms, cv::solve LU, solvePoly Durand-Kerner)",
                       "parallelism": f"hypothesis-sharded dp{world}"},
            "kernels": {"mcv_e_generate": {"avg_launch_ms": g_ms, "launches": gl},
                        "mcv_e_verify": {"avg_launch_ms": v_ms, "launches": vl}},
            "roofline": {"bound": "fp32-valu", "achieved": e_tf, "peak": FP32_PEAK_TF, "unit": "TFLOP/s",
                         "frac": e_tf / FP32_PEAK_TF,
                         "traffic": load_traffic("mcv_e_verify_pk", f"{n}x{hyps}"), "kernel": "mcv_e_verify_pk",
                         "avg_launch_ms": v_ms, "launches": vl, "models_per_launch": models,
                         "model": f"{SAMPSON_FLOPS_PER_EVAL} (fp64-definition) flops per (model, correspondence); "
                                  "certified packed-fp32 prefilter, fp64 only for undecided lanes",
                         "hbm": {"effective_GBps": alg_bytes / (v_ms * 1e-3) / 1e9,
                                 "algorithmic_bytes_per_launch": alg_bytes, "peak": HBM_PEAK_GBPS},
                         "issue": measured_issue("mcv_e_verify", f"{n}x{hyps}", n * models / (v_ms * 1e-3)) or
                                  {"achieved": n * models / (v_ms * 1e-3), "peak": issue_peak(SPK_CYC_PER_WAVE_EVAL),
                                   "unit": "evaluations/s",
                                   "frac": n * models / (v_ms * 1e-3) / issue_peak(SPK_CYC_PER_WAVE_EVAL),
                                   "model": f"certified packed-fp32 Sampson prefilter: {SPK_CYC_PER_WAVE_EVAL} SIMD "
                                            "cycles per 64 (model, correspondence) at 2.4 GHz"}},
            "result": {"best_count": result["count"], "best_slot": result["slot"],
                       "final_count": result["final_count"]},
        }
        if world == 1 and not args.no_cpu_baseline:
            sys.path.insert(0, str(ROOT / "tests"))
            import _oracle as O
            line["cpu_baseline"] = cpu_baseline_e(O.pack_e(a, b, E_FOCAL, E_PP), args.cpu_seconds)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    plan.close()


def cpu_baseline_p(img, W, K, d, target_s: float, kind: int = 1):
    sys.path.insert(0, str(ROOT / "tests"))
    import numpy as np
    import _oracle as O
    pts8, c8 = O.pack_pnp(img, W), O.cam8(K, d)
    thr2 = float(np.float32(P_THR_PX * P_THR_PX))
    threads = cpu_threads()
    t = time.perf_counter()
    O.pnp_counts(pts8, c8, P_SEED, 0, 4 * threads, thr2, False, threads, kind=kind)
    cal = (time.perf_counter() - t) / (4 * threads)
    sample = max(4 * threads, int(target_s / max(cal, 1e-6)))
    t = time.perf_counter()
    O.pnp_counts(pts8, c8, P_SEED, 0, sample, thr2, False, threads, kind=kind)
    el = time.perf_counter() - t
    solver = "4-pt AP3P" if kind in (2, 5) else "5-pt EPnP"
    return {"value": sample / el, "unit": "hypotheses/s", "cores": threads, "kind": "port", "host": host_cpu(),
            "sample": f"{sample} hypotheses x {img.shape[0]} correspondences ({solver} sample+solve, projectPoints "
                      f"fp32 error count), oracle/oracle_pnp.c + oracle_epnp.c, OpenMP {threads} threads, {el:.1f} s"}


def bench_pnp(args, world, rank, dev):
    """PnP-RANSAC (the cvSolvePnPRansac path): a step = one solvePnPRansac call over a fixed
    hypothesis budget (AP3P hypotheses, projectPoints sweep with distortion) on HBM-resident 2D-3D
    correspondences, sharded over ranks with one all-reduce, then mask + LM refit on the inliers."""
    import ctypes as C
    import numpy as np
    import torch
    import torch.distributed as dist
    from minicv_amd import native as NL, opencv, synthetic as S
    from minicv_amd import device as D
    from minicv_amd import dist as MD

    n = args.n if args.n != N_CORR else P_N_CORR
    hyps = args.hyps if args.hyps != HYPS_PER_GPU else P_HYPS_TOTAL // world
    total = hyps * world
    img, W, inl, K, d, R, t = S.pnp_problem(n, seed=P_SEED, outlier_frac=0.5, sigma=0.5,
                                            dist=[-0.12, 0.03, 0.001, -0.002])
    pts = D.pack_pnp_tensor(img, W, dev)
    plan = D.RansacPlan(NL.MODEL_PNP, n, hyps)
    plan.set_camera(K, d)
    cfg = opencv.RansacParams(threshold=P_THR_PX, confidence=0.99, max_iters=total, seed=P_SEED,
                              fixed_iters=True, fused_error=args.fused, fast_minimal=args.fast_minimal).to_c()
    kind = opencv.SOLVER_KIND[args.pnp_kind]
    cfg.pnpKind = kind
    key = torch.zeros(2, dtype=torch.int64, device=dev)
    mask = torch.zeros(n, dtype=torch.uint8, device=dev)
    red = torch.zeros(2, dtype=torch.int64, device=dev)

    def evaluate(begin, count):
        plan.evaluate(pts, n, cfg, begin, count, key)
        k = key.cpu()
        return int(k[0]), int(k[1])

    def allreduce_max(vals):
        if world == 1:
            return vals
        red.copy_(torch.tensor(vals, dtype=torch.int64))
        dist.all_reduce(red, op=dist.ReduceOp.MAX)
        return [int(v) for v in red.cpu()]

    result = {}

    def step():
        cnt, idx, _ = MD.global_best(evaluate, total, rank, world, allreduce_max)
        if idx < 0:
            raise RuntimeError("no model found")
        m = (C.c_double * 9)()
        fc = NL.lib().mcvRansacFinalize(plan._p, pts.data_ptr(), n, C.addressof(cfg), idx, m, mask.data_ptr(),
                                        D._stream_handle())
        NL.check(fc > 0, "mcvRansacFinalize")
        result.update(count=cnt, idx=idx, final_count=fc, pose=list(m[:6]))

    for _ in range(args.warmup):
        step()
    NL.lib().mcvProfileReset()
    NL.lib().mcvProfileEnable(1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    NL.lib().mcvProfileEnable(0)
    vms = C.c_double(0)
    vl = NL.lib().mcvProfileRead(b"pnp_verify", C.addressof(vms))
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    if rank == 0:
        v_ms = vms.value / max(vl, 1)
        p_bytes = 20.0 * n * hyps                # PnpPoint {X, Y, Z, u, v} f32 per (hypothesis, correspondence)
        p_fl = P_FLOPS_PER_EVAL * n * hyps / (v_ms * 1e-3) / 1e12
        evals_s = n * hyps / max(v_ms * 1e-3, 1e-12)
        common = {"traffic": load_traffic("mcv_pnp_verify", f"{n}x{hyps}"), "kernel": "mcv_pnp_verify",
                  "avg_launch_ms": v_ms, "launches": vl,
                  "hbm": {"effective_GBps": p_bytes / (v_ms * 1e-3) / 1e9,
                          "algorithmic_bytes_per_launch": p_bytes, "peak": HBM_PEAK_GBPS}}
        # default: the certified packed-fp32 sweep (mcv_pnp_verify_pk) decides the fp64 test, so the fp32
        # vector roof binds
        roof_pk = {"bound": "fp32-valu", "achieved": p_fl, "peak": FP32_PEAK_TF, "unit": "TFLOP/s",
                   "frac": p_fl / FP32_PEAK_TF, **common,
                   "model": f"{P_FLOPS_PER_EVAL} (fp64-definition) flops per (hypothesis, correspondence), a "
                            "division counted as one; decided by the certified packed-fp32 prefilter (pnp_pk.h)",
                   "issue": measured_issue("mcv_pnp_verify", f"{n}x{hyps}", evals_s) or
                            {"achieved": evals_s, "peak": issue_peak(PPK_CYC_PER_WAVE_EVAL), "unit": "evaluations/s",
                             "frac": evals_s / issue_peak(PPK_CYC_PER_WAVE_EVAL),
                             "model": f"certified packed-fp32 projection + bound: {PPK_CYC_PER_WAVE_EVAL} SIMD "
                                      "cycles per 64 (pose, point) at 2.4 GHz"}}
        line = {
            "metric": f"RANSAC hypotheses/sec, solvePnPRansac {args.pnp_kind} (cvSolvePnPRansac path) @20k corrs",
            "value": total * args.steps / el, "unit": "hypotheses/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded 2D-3D problem after Program.fs:8-24, 50% outliers, sigma 0.5 px, k1 k2 p1 p2)",
            "config": {"workload": f"solvePnPRansac {args.pnp_kind} ({'4-pt AP3P' if kind in (2, 5) else '5-pt EPnP'}"
                                   f" minimal sets), {n} correspondences x {total} hypotheses per call sharded over "
                                   f"{world} GPU(s) + {'LM' if kind == 0 else 'EPnP'} inlier solve",
                       "correspondences": n, "solver_kind": kind,
                       "minimal_solver": ("AP3P Rolle-bracket real roots (opt-in MCV_FLAG_FAST_MINIMAL)" if args.fast_minimal
                                          else "AP3P ap3p.cpp Ferrari + polish") if kind in (2, 5) else "EPnP-5",
                       "hypotheses_total": total, "threshold_px": P_THR_PX,
                       "parallelism": f"hypothesis-sharded dp{world}"},
            "kernels": {"mcv_pnp_verify": {"avg_launch_ms": v_ms, "launches": vl,
                                           "evaluations_per_s": n * hyps / max(v_ms * 1e-3, 1e-12)}},
            "roofline": roof_pk,
            "result": {"best_count": result["count"], "best_hyp": result["idx"],
                       "final_count": result["final_count"], "true_inliers": int(inl.sum())},
        }
        line["cpu_baseline"] = (cpu_baseline_p(img, W, K, d, args.cpu_seconds, kind)
                                if world == 1 and not args.no_cpu_baseline else None)
        print(json.dumps(line), flush=True)
    plan.close()


S_N_OBS = 20_000              # CameraPose.findScaled: observations per call (2 N candidates)
S_SEED = 11
S_FLOPS_PER_TERM = 30         # per (candidate, observation): 28 fp64 add/sub/mul + 2 divisions


def bench_scaled(args):
    """CameraPose.findScaled (the managed O(N^2) scale search, on the GPU behind cvFindScaledPose):
    a step = one call on HBM-resident observations: 2 N candidate scales, each verified against all
    N observations, then the first-minimum selection. Ranks run independent replicas (the path has
    no exchange step; weak scaling)."""
    import ctypes as C
    import numpy as np
    import torch
    import torch.distributed as dist
    from minicv_amd import native as NL, synthetic as S

    world, rank, dev = dist_setup(torch, dist)
    n = args.n if args.n != N_CORR else S_N_OBS
    src, pose, W, O, inl = S.scaled_problem(n, seed=S_SEED, outlier_frac=0.3, sigma=1e-3, true_scale=2.5)
    Wd = torch.from_numpy(np.ascontiguousarray(W)).to(dev)
    Od = torch.from_numpy(np.ascontiguousarray(O)).to(dev)
    cam = src.to_c()
    R = NL.M33d()
    R.M[:] = pose.Rotation.reshape(9)
    t = NL.V3d(*pose.Translation)
    cost, sc = C.c_double(0), C.c_double(0)
    stream = torch.cuda.current_stream().cuda_stream
    res = {}

    def step():
        k = NL.lib().mcvFindScaledPoseDevice(C.addressof(cam), Wd.data_ptr(), Od.data_ptr(), n, C.addressof(R),
                                             C.addressof(t), C.addressof(cost), C.addressof(sc), stream)
        NL.check(k >= 0, "mcvFindScaledPoseDevice")
        res.update(candidates=k, cost=cost.value, scale=sc.value)

    for _ in range(args.warmup):
        step()
    NL.lib().mcvProfileReset()
    NL.lib().mcvProfileEnable(1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    NL.lib().mcvProfileEnable(0)
    kms = C.c_double(0)
    launches = NL.lib().mcvProfileRead(b"scaled_costs", C.addressof(kms))
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    if rank == 0:
        avg_ms = kms.value / max(launches, 1)
        cands = 2 * n
        terms = cands * n
        tf = S_FLOPS_PER_TERM * terms / (avg_ms * 1e-3) / 1e12
        line = {
            "metric": "CameraPose.findScaled candidate scales/sec (2 N candidates x N observations)",
            "value": world * cands * args.steps / el, "unit": "candidates/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded lookAt camera + relative pose, 30% outlier observations, sigma 1e-3)",
            "config": {"workload": f"findScaled, {n} observations -> {cands} candidate scales, replicas on {world} "
                                   f"GPU(s)", "observations": n, "parallelism": f"replicas x{world}"},
            "roofline": {"bound": "fp64-valu (unfused: the managed code's op-by-op arithmetic)", "achieved": tf,
                         "peak": FP64_NOFMA_PEAK_TF, "unit": "TFLOP/s", "frac": tf / FP64_NOFMA_PEAK_TF,
                         "peak_fma": FP64_PEAK_TF, "frac_fma": tf / FP64_PEAK_TF,
                         "traffic": load_traffic("mcv_scaled_costs", f"{n}"), "kernel": "mcv_scaled_costs",
                         "avg_launch_ms": avg_ms, "launches": launches,
                         "model": f"{S_FLOPS_PER_TERM} fp64 FLOP per (candidate, observation), a division "
                                  "counted as one", "terms_per_launch": terms},
            "result": {"evaluated_candidates": res["candidates"], "cost": res["cost"], "scale": res["scale"]},
        }
        if world == 1 and not args.no_cpu_baseline:
            sys.path.insert(0, str(ROOT / "tests"))
            import _oracle as O_
            threads = cpu_threads()
            cam14 = np.concatenate([src.location, src.forward, src.up, src.right, src.focal])
            t1 = time.perf_counter()
            O_.scaled_costs_sample(cam14, W, O, pose.Rotation, pose.Translation, threads, threads)
            cal = (time.perf_counter() - t1) / threads
            sample = int(min(cands, max(threads, args.cpu_seconds / max(cal, 1e-9))))
            t1 = time.perf_counter()
            O_.scaled_costs_sample(cam14, W, O, pose.Rotation, pose.Translation, sample, threads)
            ct = time.perf_counter() - t1
            line["cpu_baseline"] = {"value": sample / ct, "unit": "candidates/s", "cores": threads, "kind": "port",
                                    "host": host_cpu(),
                                    "sample": f"{sample} candidates x {n} observations, oracle/oracle_scaled.c, "
                                              f"OpenMP {threads} threads, {ct:.1f} s"}
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
