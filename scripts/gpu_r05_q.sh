#!/bin/bash
# Round 5: kernel breakdown of the cfg5 L2 step and the Hamming step.
source scripts/gpu_step.sh
cd /tmp && export TMPDIR=/tmp
step prof_l2 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_l2_q" -o run --output-format csv -- python3 "$R/bench.py" --workload l2 --steps 5 --warmup 1 --no-cpu-baseline --no-secondary
