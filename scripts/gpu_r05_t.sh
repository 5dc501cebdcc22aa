#!/bin/bash
# Round 5 screen: EPnP kernel split (mtm / sweeps / tail / betas / pose) times.
source scripts/gpu_step.sh
step tests_t 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pnp.py -k "epnp or EPNP or full or counts"
cd /tmp && export TMPDIR=/tmp
step prof_t 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_pnp_t" -o run --output-format csv -- python3 "$R/bench.py" --workload pnp --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
