#!/bin/bash
# Round 5 screen (experiment builds): PnP verify poses per wave x waves per EU: 1 = 2 x 6, 2 = 2 x 7,
# 3 = 4 x 4, 4 = 3 x 6, against 3 x 5.
source scripts/gpu_step.sh
for i in 1 2; do
step p_base$i 300 python bench.py --workload pnp --steps 4 --warmup 1 --no-cpu-baseline --no-secondary
for n in 1 2 3 4; do
MINICV_NATIVE_LIB=$R/libs/exp/$n/libMiniCVNative.so step p_v${n}_$i 300 python bench.py --workload pnp --steps 4 --warmup 1 --no-cpu-baseline --no-secondary
done
done
