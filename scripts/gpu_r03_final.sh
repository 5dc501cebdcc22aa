#!/bin/bash
# Round-3 evidence: full GPU suite, every bench line (+ fused homography, AP3P PnP), rocprofv3
# kernel-trace stats per workload and the PMC traffic passes. Stops at the first failing GPU step.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {   # name timeout cmd...
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "$R/gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -2 "$R/gpurun_out/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
# PARTS: any of t (tests), b (benches), p (profiles); default all
PARTS=${PARTS:-tbp}
if [[ $PARTS == *t* ]]; then
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread
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
fi
[[ $PARTS == *p* ]] || exit 0
cd /tmp && export TMPDIR=/tmp
for w in homography fundamental essential pnp hamming l2 scaled; do
    step prof_$w 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
done
for w in homography fundamental essential pnp hamming l2 scaled; do
    step pmc_fetch_$w 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
    step pmc_write_$w 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
done
# SQ passes: measured VALU instructions per evaluation / VALU busy share of each workload's sweep
for w in homography fundamental essential pnp; do
    step pmc_sq_$w 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
        --output-format csv -d "$R/gpurun_out/pmc_sq_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
done
step pmc_lds_homography 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --output-format csv -d "$R/gpurun_out/pmc_lds_homography" -o run -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
