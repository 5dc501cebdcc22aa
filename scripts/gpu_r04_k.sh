#!/bin/bash
# E verify at 2^20 hypotheses: one point chunk (no partial-count atomics) vs the 50k-point chunks; WRITE_SIZE per launch.
set -u
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in "c50k 50000" "c1 1000000"; do
    set -- $v
    MCV_E_CHUNK=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_echunk_$1" -o run -- \
        python3 "$R/bench.py" --workload essential --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > "$R/gpurun_out/echunk_$1.log" 2>&1 || exit 1
    MCV_E_CHUNK=$2 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_echunk_$1" -o run -- \
        python3 "$R/bench.py" --workload essential --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > /dev/null 2>&1 || exit 1
done
