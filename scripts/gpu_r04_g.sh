#!/bin/bash
# L2 at the query-sharded ranks' shares (adaptive train chunks): exactness tests, share timings, kernel breakdown.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matchers.py -k "l2" > gpurun_out/l2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/l2_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/exp/l2_shard_timing.py > gpurun_out/l2_share.log 2>&1
rc=$?; cat gpurun_out/l2_share.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_l2share" -o run -- \
    python3 "$R/scripts/exp/l2_shard_timing.py" > "$R/gpurun_out/prof_l2share.log" 2>&1
rc=$?; [ $rc -ne 0 ] && exit $rc
f=$(find "$R/gpurun_out/prof_l2share" -name '*kernel_stats.csv' | head -1); cut -d, -f1-5 "$f" | head -20
