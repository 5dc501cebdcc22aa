#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r02s
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_scaled.py \
    > gpurun_out/r02s/pytest_scaled.log 2>&1 || exit 2
timeout -k 10 200 python bench.py --workload scaled --steps 5 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r02s/bench_scaled.json 2> gpurun_out/r02s/bench_scaled.err || exit 3
