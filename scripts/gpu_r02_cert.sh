#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r02i
export PYTHONUNBUFFERED=1
MCV_HCERT_VARIANT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_selftest.py tests/test_gpu_homography.py > gpurun_out/r02i/pytest_v1.log 2>&1 || exit 2
for v in 1 2 3 4 5 8 90 91; do
  MCV_HCERT_VARIANT=$v timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline \
      > gpurun_out/r02i/bench_h_v$v.json 2> gpurun_out/r02i/bench_h_v$v.err || exit 3
done
