#!/bin/bash
# F / E verify at 2^20 hypotheses with 8 per-XCD point chunks (L2-resident slices) vs the default; time + FETCH/WRITE.
set -u
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
run() {   # name workload env...
    local name=$1 w=$2; shift 2
    env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_xc_$name" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > "$R/gpurun_out/xc_$name.log" 2>&1 || exit 1
    env "$@" timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_xcf_$name" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > /dev/null 2>&1 || exit 1
    env "$@" timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_xcw_$name" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > /dev/null 2>&1 || exit 1
}
run f_def fundamental MCV_F_WAVES=65536
run f_c8 fundamental MCV_F_WAVES=1048576
run e_c8 essential MCV_E_CHUNK=12500
