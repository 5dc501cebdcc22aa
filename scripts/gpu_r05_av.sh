#!/bin/bash
# Round 5: L2 GEMM epilogue priority vs HEAD, same box, alternating three times.
source scripts/gpu_step.sh
for i in 1 2 3; do
step l2_new$i 300 python bench.py --workload l2 --steps 20 --warmup 2 --no-cpu-baseline --no-secondary
MINICV_NATIVE_LIB=$R/libs/old/libMiniCVNative.so step l2_old$i 300 python bench.py --workload l2 --steps 20 --warmup 2 --no-cpu-baseline --no-secondary
done
