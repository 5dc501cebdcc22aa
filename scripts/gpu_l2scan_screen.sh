#!/bin/bash
# Exact-scan grid screen: matcher tests, then a kernel-trace profile of the L2 bench per
# MCV_L2_SCAN_BLOCKS value. Stops at the first failing GPU step.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_matchers.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_l2scan.log 2>&1 || { tail -5 gpurun_out/pytest_l2scan.log; exit 1; }
tail -1 gpurun_out/pytest_l2scan.log
cd /tmp && export TMPDIR=/tmp
for b in ${BLOCKS:-1024 2048 4096}; do
    MCV_L2_SCAN_BLOCKS=$b timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$R/gpurun_out/prof_scan_$b" -o run -- python3 "$R/bench.py" --workload l2 --steps 5 --warmup 2 \
        --no-cpu-baseline > "$R/gpurun_out/prof_scan_$b.log" 2>&1 || { echo "blocks $b failed"; exit 2; }
    echo "blocks $b ok"
done
