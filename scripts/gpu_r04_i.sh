#!/bin/bash
# experiment: wall-clock stamps inside the exact scan (debug build)
set -u
timeout -k 10 120 python3 scripts/exp/l2_shard_timing.py > gpurun_out/l2_stamps.log 2>&1 || exit 1
