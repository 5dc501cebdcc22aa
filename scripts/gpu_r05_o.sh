#!/bin/bash
# Round 5: Hamming GEMM form folds its chunks in the last block (release-only fence per block).
source scripts/gpu_step.sh
step tests_o 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_matchers.py
step bench_hamming 300 python bench.py --workload hamming --steps 50 --warmup 5 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
step prof_ham 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_ham_o" -o run --output-format csv -- python3 "$R/bench.py" --workload hamming --steps 20 --warmup 2 --no-cpu-baseline --no-secondary
