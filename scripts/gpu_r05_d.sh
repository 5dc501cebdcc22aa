#!/bin/bash
# Round 5: L2 prep with atomic slots + refine prefetch: matcher tests, share timing, kernel trace.
source scripts/gpu_step.sh
step tests_d 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_matchers.py tests/test_gpu_pipeline.py
step l2_share 200 python scripts/exp/l2_shard_timing.py
cat gpurun_out/l2_share.log
cd /tmp && export TMPDIR=/tmp
step prof_l2share 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_l2share" -o run -- python3 "$R/scripts/exp/l2_shard_timing.py"
