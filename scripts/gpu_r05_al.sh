#!/bin/bash
# Round 5: PnP bench line and rank shares after the EPnP pass change.
source scripts/gpu_step.sh
step bench_pnp 300 python bench.py --workload pnp --steps 5 --warmup 2 --cpu-seconds 8
step rank_share_pnp 600 python scripts/exp/rank_share_timing.py pnp
cd /tmp && export TMPDIR=/tmp
step prof_pnp 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_pnp" -o run -- \
    python3 "$R/bench.py" --workload pnp --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
