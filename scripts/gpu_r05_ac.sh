#!/bin/bash
# Round 5 screen: L2 f16 GEMM staged by LDS-DMA (swizzled unpadded tile image) vs register staging (HEAD).
source scripts/gpu_step.sh
step test_match 300 python -u -m pytest tests/test_gpu_matchers.py -x -q --timeout 120 --timeout-method thread
for i in 1 2; do
step l2_new$i 300 python bench.py --workload l2 --steps 20 --warmup 2 --no-cpu-baseline --no-secondary
MINICV_NATIVE_LIB=$R/libs/old/libMiniCVNative.so step l2_old$i 300 python bench.py --workload l2 --steps 20 --warmup 2 --no-cpu-baseline --no-secondary
done
