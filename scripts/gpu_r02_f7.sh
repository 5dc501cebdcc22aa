#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r02f
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fundamental.py \
    > gpurun_out/r02f/pytest_f.log 2>&1 || exit 2
