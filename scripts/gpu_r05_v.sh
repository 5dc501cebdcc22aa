#!/bin/bash
# Round 5: JacobiSVDImpl_ rotation with the refined-reciprocal quotients and unscaled sqrt; PnP verify
# at 2 poses per wave (interleaved chains).
source scripts/gpu_step.sh
step tests_v 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_selftest.py tests/test_gpu_pnp.py tests/test_gpu_fundamental.py
step bench_pnp 300 python bench.py --workload pnp --steps 5 --warmup 2 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
step prof_v 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_pnp_v" -o run --output-format csv -- python3 "$R/bench.py" --workload pnp --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
