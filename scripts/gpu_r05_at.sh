#!/bin/bash
# Round 5 screen (experiment builds, -DMCV_EXP_PRIO=N): s_setprio 1 around the L2 GEMM's MFMA block (1)
# or around its epilogue (2), with the LDS-DMA staging.
source scripts/gpu_step.sh
for i in 1 2; do
step l2_base$i 300 python bench.py --workload l2 --steps 20 --warmup 2 --no-cpu-baseline --no-secondary
for n in 1 2; do
MINICV_NATIVE_LIB=$R/libs/exp/$n/libMiniCVNative.so step l2_v${n}_$i 300 python bench.py --workload l2 --steps 20 --warmup 2 --no-cpu-baseline --no-secondary
done
done
