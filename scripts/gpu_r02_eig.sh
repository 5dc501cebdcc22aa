#!/bin/bash
# H / F minimal solvers (cv::eigen default, elimination opt-in): GPU parity tests, benches, kernel stats.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {   # name timeout cmd...
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "$R/gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -3 "$R/gpurun_out/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step pytest_eig 600 python -u -m pytest tests/test_gpu_homography.py tests/test_gpu_fundamental.py tests/test_gpu_pipeline.py tests/test_gpu_multishard.py -m gpu -x -q --timeout 300 --timeout-method thread
step bench_h 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
step bench_h_fast 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --fast-minimal
step bench_f 300 python bench.py --workload fundamental --steps 5 --warmup 1 --no-cpu-baseline
