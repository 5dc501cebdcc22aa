#!/bin/bash
# Round 5: L2 GEMM with three independent accumulator chains.
source scripts/gpu_step.sh
step tests_r 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_matchers.py -k "l2 or matchers"
step bench_l2 300 python bench.py --workload l2 --steps 10 --warmup 2 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
step prof_l2 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_l2_r" -o run --output-format csv -- python3 "$R/bench.py" --workload l2 --steps 5 --warmup 1 --no-cpu-baseline --no-secondary
