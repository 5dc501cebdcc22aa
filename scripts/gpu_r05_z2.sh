#!/bin/bash
# Round 5: L2 rank shares timed back to back (as bench.py's loop) and a kernel trace of the 8-rank share.
source scripts/gpu_step.sh
step rank_share_l2 300 python scripts/exp/rank_share_timing.py l2
cd /tmp && export TMPDIR=/tmp
step prof_l2_share8 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_l2_share8" -o run -- \
    python3 "$R/scripts/exp/l2_share_prof.py" 8
