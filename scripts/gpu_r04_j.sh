#!/bin/bash
# Four-lane eigen generate (MCV_EIG_Q4): H tests bit-exact under the quad form; generate timings per block size.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
MCV_EIG_Q4=40 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_homography.py > gpurun_out/q4_tests.log 2>&1
rc=$?; tail -3 gpurun_out/q4_tests.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for v in 0 32 40 64; do
    MCV_EIG_Q4=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_q4_$v" -o run -- \
        python3 "$R/bench.py" --workload homography --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/q4_$v.log" 2>&1 || exit 1
    echo "== q4=$v"; grep -h "generate" $(find "$R/gpurun_out/prof_q4_$v" -name '*kernel_stats.csv') | cut -d, -f1-4
done
