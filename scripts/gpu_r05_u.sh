#!/bin/bash
# Round 5: PnP verify with the K pose chains in one basic block.
source scripts/gpu_step.sh
step tests_u 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pnp.py
step bench_pnp 300 python bench.py --workload pnp --steps 5 --warmup 2 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
step prof_u 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_pnp_u" -o run --output-format csv -- python3 "$R/bench.py" --workload pnp --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
