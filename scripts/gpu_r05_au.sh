#!/bin/bash
# Round 5: L2 GEMM with epilogue priority (parity + bench), and the same priority split screened on the
# Hamming GEMM (experiment build 1).
source scripts/gpu_step.sh
step test_match 300 python -u -m pytest tests/test_gpu_matchers.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread
step l2_new 300 python bench.py --workload l2 --steps 20 --warmup 2 --no-cpu-baseline --no-secondary
for i in 1 2; do
step h_base$i 300 python bench.py --workload hamming --steps 200 --warmup 20 --no-cpu-baseline --no-secondary
MINICV_NATIVE_LIB=$R/libs/exp/1/libMiniCVNative.so step h_v1_$i 300 python bench.py --workload hamming --steps 200 --warmup 20 --no-cpu-baseline --no-secondary
done
