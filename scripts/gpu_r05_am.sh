#!/bin/bash
# Round 5 screen (experiment builds, -DMCV_EXP_H=N): the certified H sweep with 4 x 1 / 5 x 1 / 4 x 2
# (models x points a trip) against 6 x 1.
source scripts/gpu_step.sh
for i in 1 2; do
step h_base$i 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-secondary
for n in 1 2 3; do
MINICV_NATIVE_LIB=$R/libs/exp/$n/libMiniCVNative.so step h_v${n}_$i 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-secondary
done
done
