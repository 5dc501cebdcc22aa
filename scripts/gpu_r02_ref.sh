#!/bin/bash
# Round-2: reference-path exports (solveAp3p Ferrari, cvFivePoint solvePoly) + PnP / essential GPU parity.
set -o pipefail
mkdir -p gpurun_out/r02r
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pnp.py \
    tests/test_gpu_essential.py > gpurun_out/r02r/pytest_pnp_e.log 2>&1 || exit 2
