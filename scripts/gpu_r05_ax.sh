#!/bin/bash
# Round 5: L2 refine with eight partials in flight per query vs HEAD: parity, rank shares (same box,
# alternating), kernel trace at the 8-rank share.
source scripts/gpu_step.sh
step test_match 300 python -u -m pytest tests/test_gpu_matchers.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread
for i in 1 2; do
step share_new$i 300 python scripts/exp/rank_share_timing.py l2
MINICV_NATIVE_LIB=$R/libs/old/libMiniCVNative.so step share_old$i 300 python scripts/exp/rank_share_timing.py l2
done
cd /tmp && export TMPDIR=/tmp
for n in 1 8; do
step prof_rf_$n 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_rf_$n" -o run -- \
    python3 "$R/scripts/exp/l2_share_prof.py" $n
done
