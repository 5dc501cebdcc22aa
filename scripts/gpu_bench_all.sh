#!/bin/bash
# Run the GPU test suite and every bench workload on one MI355X (used through gpurun).
# Stops at the first GPU step that times out / faults (exit status > 1).
set -u
mkdir -p gpurun_out
step() {   # name timeout cmd...
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log"
    if [ $rc -gt 1 ]; then exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench_homography 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 8
step bench_fundamental 300 python bench.py --workload fundamental --steps 5 --warmup 1 --cpu-seconds 8
step bench_hamming 300 python bench.py --workload hamming --steps 20 --warmup 3
step bench_l2 300 python bench.py --workload l2 --steps 5 --warmup 2
step bench_essential 300 python bench.py --workload essential --steps 5 --warmup 2 --cpu-seconds 8
step bench_pnp 300 python bench.py --workload pnp --steps 5 --warmup 2 --cpu-seconds 8
step bench_scaled 300 python bench.py --workload scaled --steps 5 --warmup 2 --cpu-seconds 8
