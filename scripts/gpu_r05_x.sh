#!/bin/bash
# Round 5 screen: L2 GEMM stream-K partition vs the (query block, chunk) grid, same box, alternating.
source scripts/gpu_step.sh
for i in 1 2; do
step bench_l2_new$i 300 python bench.py --workload l2 --steps 20 --warmup 2 --no-cpu-baseline
MCV_EXP_L2_OLD=1 step bench_l2_old$i 300 python bench.py --workload l2 --steps 20 --warmup 2 --no-cpu-baseline
done
