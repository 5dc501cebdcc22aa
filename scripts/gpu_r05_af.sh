#!/bin/bash
# Round 5: F parity with 3 model pairs per wave (the new default), and an E verify screen
# (experiment builds, -DMCV_EXP_E=N: 1 = 3 pairs x 1 point, 2 = 2 x 2, 3 = 2 x 1; default 3 x 2).
source scripts/gpu_step.sh
step test_f 600 python -u -m pytest tests/test_gpu_fundamental.py -x -q --timeout 300 --timeout-method thread
for i in 1 2; do
step e_base$i 300 python bench.py --workload essential --steps 4 --warmup 1 --no-cpu-baseline --no-secondary
for n in 1 2 3; do
MINICV_NATIVE_LIB=$R/libs/exp/$n/libMiniCVNative.so step e_v${n}_$i 300 python bench.py --workload essential --steps 4 --warmup 1 --no-cpu-baseline --no-secondary
done
done
