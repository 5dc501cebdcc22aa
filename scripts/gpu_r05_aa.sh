#!/bin/bash
# Round 5 screen: L2 refine with 16 lanes per query and the exact merge's batched loads vs HEAD, same box.
source scripts/gpu_step.sh
step test_match 300 python -u -m pytest tests/test_gpu_matchers.py -x -q --timeout 120 --timeout-method thread
for i in 1 2; do
step share_new$i 300 python scripts/exp/rank_share_timing.py l2
MINICV_NATIVE_LIB=$R/libs/old/libMiniCVNative.so step share_old$i 300 python scripts/exp/rank_share_timing.py l2
done
step bench_l2_new 300 python bench.py --workload l2 --steps 20 --warmup 2 --no-cpu-baseline
MINICV_NATIVE_LIB=$R/libs/old/libMiniCVNative.so step bench_l2_old 300 python bench.py --workload l2 --steps 20 --warmup 2 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
step prof_l2_share8 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_l2_share8" -o run -- \
    python3 "$R/scripts/exp/l2_share_prof.py" 8
