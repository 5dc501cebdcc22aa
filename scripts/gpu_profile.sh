#!/bin/bash
# rocprofv3 kernel-trace stats for each bench workload, then PMC counter passes (separate runs,
# --kernel-trace only beside --pmc) for the headline sweep. Output under gpurun_out/prof_*.
set -u
R=$PWD
cd /tmp && export TMPDIR=/tmp
run() {   # name timeout args...
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "$R/gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$R/gpurun_out/$name.log"; exit $rc; fi
}
for w in homography fundamental essential pnp hamming l2 scaled; do
    run prof_$w 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 5 --warmup 2 --no-cpu-baseline
done
# PMC passes (one counter per run) on each BASELINE workload's bench, then SQ counters of the H sweep
for w in homography fundamental essential pnp hamming l2 scaled; do
    run pmc_fetch_$w 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline
    run pmc_write_$w 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline
done
run pmc_sq 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/pmc_sq" -o run -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline
