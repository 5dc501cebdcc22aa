#!/bin/bash
# Round 5 screen (experiment builds, -DMCV_EXP_F=N): F verify with 3 model pairs per wave (P = 1 / 2:
# four waves per SIMD) and 2 pairs (P = 2: five) against 4 pairs (three waves per SIMD).
source scripts/gpu_step.sh
for i in 1 2; do
step f_base$i 300 python bench.py --workload fundamental --steps 4 --warmup 1 --no-cpu-baseline --no-secondary
for n in 1 2 3; do
MINICV_NATIVE_LIB=$R/libs/exp/$n/libMiniCVNative.so step f_v${n}_$i 300 python bench.py --workload fundamental --steps 4 --warmup 1 --no-cpu-baseline --no-secondary
done
done
