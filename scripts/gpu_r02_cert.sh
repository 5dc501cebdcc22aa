#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r02k
export PYTHONUNBUFFERED=1
MCV_HCERT_VARIANT=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_selftest.py tests/test_gpu_homography.py > gpurun_out/r02k/pytest_v3.log 2>&1 || exit 2
for t in 0.000244140625 0.00048828125 0.0009765625; do
for v in 3 8 2; do
  MCV_HCERT_T=$t MCV_HCERT_VARIANT=$v timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline \
      > gpurun_out/r02k/bench_h_v${v}_t$t.json 2> gpurun_out/r02k/bench_h_v${v}_t$t.err || exit 3
done
done
