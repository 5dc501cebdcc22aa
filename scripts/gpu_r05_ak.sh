#!/bin/bash
# Round 5: EPnP inlier passes with 128-point tiles: PnP parity, the 8-rank share's kernel trace, bench.
source scripts/gpu_step.sh
step test_pnp 600 python -u -m pytest tests/test_gpu_pnp.py -x -q --timeout 300 --timeout-method thread
step bench_pnp_share8 300 python bench.py --workload pnp --hyps 131072 --steps 6 --warmup 2 --no-cpu-baseline --no-secondary
step bench_pnp 300 python bench.py --workload pnp --steps 5 --warmup 2 --cpu-seconds 8
cd /tmp && export TMPDIR=/tmp
step prof_pnp_share8 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_pnp_share8" -o run -- \
    python3 "$R/bench.py" --workload pnp --hyps 131072 --steps 6 --warmup 2 --no-cpu-baseline --no-secondary
