#!/bin/bash
# L2 exact scan with lane-parallel exact rows: exactness tests, share timings, kernel breakdown.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matchers.py -k "l2" > gpurun_out/l2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/l2_tests.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 "$R/scripts/exp/l2_shard_timing.py" > "$R/gpurun_out/l2s_lane.log" 2>&1 || exit 1
grep '^{' "$R/gpurun_out/l2s_lane.log"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_l2s_lane" -o run -- \
    python3 "$R/scripts/exp/l2_shard_timing.py" > "$R/gpurun_out/prof_l2s_lane.log" 2>&1 || exit 1
