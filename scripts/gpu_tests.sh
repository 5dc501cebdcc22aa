#!/bin/bash
# Run the given GPU test files (default: the whole -m gpu suite) in one pytest process.
set -o pipefail
mkdir -p gpurun_out/tests
export PYTHONUNBUFFERED=1
files="${*:-tests}"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $files \
    > gpurun_out/tests/pytest.log 2>&1 || { tail -30 gpurun_out/tests/pytest.log; exit 2; }
tail -3 gpurun_out/tests/pytest.log
