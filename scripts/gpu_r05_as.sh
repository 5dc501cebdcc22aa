#!/bin/bash
# Round 5 screen (experiment builds): Hamming GEMM with one query tile per wave at four (1) / five (2)
# waves per SIMD against two query tiles at three.
source scripts/gpu_step.sh
MINICV_NATIVE_LIB=$R/libs/exp/1/libMiniCVNative.so step test_v1 300 python -u -m pytest tests/test_gpu_matchers.py -x -q -k hamming --timeout 120 --timeout-method thread
for i in 1 2; do
step h_base$i 300 python bench.py --workload hamming --steps 200 --warmup 20 --no-cpu-baseline --no-secondary
for n in 1 2; do
MINICV_NATIVE_LIB=$R/libs/exp/$n/libMiniCVNative.so step h_v${n}_$i 300 python bench.py --workload hamming --steps 200 --warmup 20 --no-cpu-baseline --no-secondary
done
done
