#!/bin/bash
# Round 5: what the 8-rank PnP share (2^17 hypotheses) is made of: kernel trace + bench line.
source scripts/gpu_step.sh
step bench_pnp_share8 300 python bench.py --workload pnp --hyps 131072 --steps 6 --warmup 2 --no-cpu-baseline --no-secondary
cd /tmp && export TMPDIR=/tmp
step prof_pnp_share8 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_pnp_share8" -o run -- \
    python3 "$R/bench.py" --workload pnp --hyps 131072 --steps 6 --warmup 2 --no-cpu-baseline --no-secondary
