#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r02e
export PYTHONUNBUFFERED=1
for v in 2 7; do
  MCV_HCERT_VARIANT=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_selftest.py tests/test_gpu_homography.py > gpurun_out/r02e/pytest_v$v.log 2>&1 || exit 2
done
for v in 2 4 7 0; do
  MCV_HCERT_VARIANT=$v timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline \
      > gpurun_out/r02e/bench_h_v$v.json 2> gpurun_out/r02e/bench_h_v$v.err || exit 3
done
for v in 2 7; do
  MCV_HCERT_NOREDO=1 MCV_HCERT_VARIANT=$v timeout -k 10 120 python scripts/exp/hcert_diag.py >> gpurun_out/r02e/diag.txt 2>&1 || exit 1
done
