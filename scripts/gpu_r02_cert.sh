#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r02j
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_matchers.py tests/test_gpu_pipeline.py > gpurun_out/r02j/pytest_m.log 2>&1 || exit 2
timeout -k 10 120 python bench.py --workload l2 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r02j/bench_l2.json 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02j/prof_l2 -o run -- python3 bench.py --workload l2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r02j/prof_l2.log 2>&1 || exit 5
