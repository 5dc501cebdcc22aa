#!/bin/bash
# Round 5 screen: Hamming GEMM with the top-2 updates pipelined one tile behind the MFMAs
# (experiment builds: 1 = three waves per SIMD with spills, 2 = two waves per SIMD) against HEAD.
source scripts/gpu_step.sh
MINICV_NATIVE_LIB=$R/libs/exp/2/libMiniCVNative.so step test_v2 300 python -u -m pytest tests/test_gpu_matchers.py -x -q -k hamming --timeout 120 --timeout-method thread
for i in 1 2; do
MINICV_NATIVE_LIB=$R/libs/old/libMiniCVNative.so step h_old$i 300 python bench.py --workload hamming --steps 200 --warmup 20 --no-cpu-baseline --no-secondary
for n in 1 2; do
MINICV_NATIVE_LIB=$R/libs/exp/$n/libMiniCVNative.so step h_v${n}_$i 300 python bench.py --workload hamming --steps 200 --warmup 20 --no-cpu-baseline --no-secondary
done
done
