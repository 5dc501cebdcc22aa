#!/bin/bash
# MFMA-filtered exact scan: matcher tests (default and forced VALU scan), rank shares, kernel breakdown.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matchers.py tests/test_gpu_pipeline.py > gpurun_out/s16_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s16_tests.log; [ $rc -ne 0 ] && exit $rc
MCV_L2_SCAN16=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matchers.py -k l2 > gpurun_out/s16_tests0.log 2>&1
rc=$?; tail -1 gpurun_out/s16_tests0.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0; do
    MCV_L2_SCAN16=$v timeout -k 10 120 python3 scripts/exp/l2_shard_timing.py > gpurun_out/l2s16_$v.log 2>&1 || exit 1
    echo "scan16=$v $(grep -h '^{' gpurun_out/l2s16_$v.log | python3 -c "import sys,json; print(' '.join('%d:%.3f' % (d['ranks'], d['ms']) for d in map(json.loads, sys.stdin)))")"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_l2s16" -o run -- \
    python3 "$R/scripts/exp/l2_shard_timing.py" > "$R/gpurun_out/prof_l2s16.log" 2>&1 || exit 1
