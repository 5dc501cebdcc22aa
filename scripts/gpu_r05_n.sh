#!/bin/bash
# Round 5: PnP verify at 5 waves per EU; Hamming merge with 8 lanes per query.
source scripts/gpu_step.sh
step tests_n 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pnp.py tests/test_gpu_matchers.py
step bench_pnp 300 python bench.py --workload pnp --steps 5 --warmup 2 --no-cpu-baseline
step bench_hamming 300 python bench.py --workload hamming --steps 50 --warmup 5 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
step prof_pnp 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_pnp_n" -o run --output-format csv -- python3 "$R/bench.py" --workload pnp --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
step prof_ham 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_ham_n" -o run --output-format csv -- python3 "$R/bench.py" --workload hamming --steps 20 --warmup 2 --no-cpu-baseline --no-secondary
