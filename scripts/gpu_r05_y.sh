#!/bin/bash
# Round 5 screen: Hamming GEMM stream-K partition vs the (query block, chunk) grid, same box, alternating.
source scripts/gpu_step.sh
step test_match 300 python -u -m pytest tests/test_gpu_matchers.py -x -q --timeout 120 --timeout-method thread
for i in 1 2; do
step bench_h_new$i 300 python bench.py --workload hamming --steps 200 --warmup 20 --no-cpu-baseline
MINICV_NATIVE_LIB=$R/libs/old/libMiniCVNative.so step bench_h_old$i 300 python bench.py --workload hamming --steps 200 --warmup 20 --no-cpu-baseline
MCV_HAM_PERCU=6 step bench_h_pc6_$i 300 python bench.py --workload hamming --steps 200 --warmup 20 --no-cpu-baseline
done
