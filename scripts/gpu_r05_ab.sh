#!/bin/bash
# Round 5 screen (experiment builds, -DMCV_EXP_L2=N): 11 = 6-wave blocks (192 queries share each staged
# train tile, 2 blocks per CU) in the f16 domain.
source scripts/gpu_step.sh
MINICV_NATIVE_LIB=$R/libs/exp/11/libMiniCVNative.so step test_v11 300 python -u -m pytest tests/test_gpu_matchers.py -x -q -k "full_size_cfg5 or medium_vs_oracle" --timeout 120 --timeout-method thread
for i in 1 2; do
step l2_base$i 300 python bench.py --workload l2 --steps 20 --warmup 2 --no-cpu-baseline --no-secondary
for n in 11; do
MINICV_NATIVE_LIB=$R/libs/exp/$n/libMiniCVNative.so step l2_v${n}_$i 300 python bench.py --workload l2 --steps 20 --warmup 2 --no-cpu-baseline --no-secondary
done
done
