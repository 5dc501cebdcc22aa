#!/bin/bash
# Round-4 closing run: F with the L2-sized point chunks (tests, kernel stats, PMC traffic / SQ), the
# traffic summary rebuilt on the box, then every bench line again so each line carries this round's
# measured traffic.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "$R/gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -1 "$R/gpurun_out/$name.log" | cut -c1-160
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step f_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fundamental.py tests/test_gpu_multishard.py
(
cd /tmp && export TMPDIR=/tmp
w=fundamental
step prof_$w 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$w" -o run -- \
    python3 "$R/bench.py" --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
step pmc_fetch_$w 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch_$w" -o run -- \
    python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
step pmc_write_$w 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write_$w" -o run -- \
    python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
step pmc_sq_$w 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
    --output-format csv -d "$R/gpurun_out/pmc_sq_$w" -o run -- \
    python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
) || exit 1
step collect 120 python3 scripts/collect_profiles.py r04
PARTS=b bash scripts/gpu_r04_final.sh
