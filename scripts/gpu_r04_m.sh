#!/bin/bash
# Essential after the single-chunk default: tests, bench line, kernel stats, PMC traffic + SQ passes.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "$R/gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -1 "$R/gpurun_out/$name.log" | cut -c1-200
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step e_tests 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_essential.py
step bench_essential 300 python bench.py --workload essential --steps 5 --warmup 2 --cpu-seconds 8
step bench_essential_fast 300 python bench.py --workload essential --steps 5 --warmup 2 --no-cpu-baseline --fast-minimal
cd /tmp && export TMPDIR=/tmp
w=essential
step prof_$w 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$w" -o run -- \
    python3 "$R/bench.py" --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
step pmc_fetch_$w 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch_$w" -o run -- \
    python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
step pmc_write_$w 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write_$w" -o run -- \
    python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
step pmc_sq_$w 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
    --output-format csv -d "$R/gpurun_out/pmc_sq_$w" -o run -- \
    python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
