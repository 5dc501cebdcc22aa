#!/bin/bash
# Round 5: AP3P fully on the device (glibc exp / log / log1p / cos / atan2 restated): PnP parity + benches.
source scripts/gpu_step.sh
step tests_pnp 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pnp.py -s -k "ap3p or AP3P or pnp"
step bench_ap3p 300 python bench.py --workload pnp --pnp-kind AP3P --steps 5 --warmup 2 --no-cpu-baseline
step bench_pnp 300 python bench.py --workload pnp --steps 5 --warmup 2 --no-cpu-baseline
