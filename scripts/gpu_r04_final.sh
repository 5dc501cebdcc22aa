#!/bin/bash
# Round-4 evidence: full GPU suite, every bench line, --gpus 2 self-launch (gloo, one device), rocprofv3
# kernel-trace stats per workload, PMC traffic passes, SQ (VALU / MFMA) passes, the H generate's
# lane-vs-quad SQ counters and the L2 rank-share timings. Stops at the first failing GPU step.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {   # name timeout cmd...
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "$R/gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -2 "$R/gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ne 0 ]; then exit $rc; fi
}
# PARTS: any of t (tests), b (benches), p (profiles), c (counters); default all
PARTS=${PARTS:-tbpc}
if [[ $PARTS == *t* ]]; then
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $PARTS == *b* ]]; then
step bench_homography 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 8
step bench_homography_fused 300 python bench.py --steps 10 --warmup 3 --fused --no-cpu-baseline
step bench_homography_fast 300 python bench.py --steps 10 --warmup 3 --fast-minimal --no-cpu-baseline
step bench_fundamental 300 python bench.py --workload fundamental --steps 5 --warmup 1 --cpu-seconds 8
step bench_hamming 300 python bench.py --workload hamming --steps 20 --warmup 3
step bench_l2 300 python bench.py --workload l2 --steps 5 --warmup 2
step bench_essential 300 python bench.py --workload essential --steps 5 --warmup 2 --cpu-seconds 8
step bench_pnp 300 python bench.py --workload pnp --steps 5 --warmup 2 --cpu-seconds 8
step bench_pnp_ap3p 300 python bench.py --workload pnp --pnp-kind AP3P --steps 5 --warmup 2 --no-cpu-baseline
step bench_essential_fast 300 python bench.py --workload essential --steps 5 --warmup 2 --no-cpu-baseline --fast-minimal
step bench_scaled 300 python bench.py --workload scaled --steps 5 --warmup 2 --cpu-seconds 8
for w in fundamental l2; do
    MCV_DIST_BACKEND=gloo step selflaunch_$w 300 python bench.py --workload $w --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline
done
step l2_share 200 python scripts/exp/l2_shard_timing.py
fi
cd /tmp && export TMPDIR=/tmp
if [[ $PARTS == *p* ]]; then
for w in homography fundamental essential pnp hamming l2 scaled; do
    step prof_$w 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
done
fi
[[ $PARTS == *c* ]] || exit 0
for w in homography fundamental essential pnp hamming l2 scaled; do
    step pmc_fetch_$w 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
    step pmc_write_$w 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
done
# SQ passes: VALU instructions per evaluation / VALU busy share of each sweep
for w in homography fundamental essential pnp; do
    step pmc_sq_$w 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
        --output-format csv -d "$R/gpurun_out/pmc_sq_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
done
# MFMA passes of the matchers' GEMM kernels
for w in hamming l2; do
    step pmc_mfma_$w 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE \
        --output-format csv -d "$R/gpurun_out/pmc_mfma_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
done
# the H generate, one lane vs four lanes per hypothesis
for v in "lane 0" "quad 40"; do
    set -- $v
    MCV_EIG_Q4=$2 step pmc_gen_$1 120 rocprofv3 --kernel-trace --kernel-include-regex "h_generate" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE \
        --output-format csv -d "$R/gpurun_out/pmc_gen_$1" -o run -- \
        python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-secondary
done
