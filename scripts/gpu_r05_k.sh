#!/bin/bash
# Round 5: F verify without L2 chunks (one count store per model): parity, bench, WRITE_SIZE; E bench.
source scripts/gpu_step.sh
step tests_k 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fundamental.py
step bench_fundamental 300 python bench.py --workload fundamental --steps 3 --warmup 1 --no-cpu-baseline
step bench_essential 300 python bench.py --workload essential --steps 3 --warmup 1 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
step pmc_write_fundamental 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write_fundamental_k" -o run -- python3 "$R/bench.py" --workload fundamental --steps 1 --warmup 1 --no-cpu-baseline --no-secondary
step pmc_fetch_fundamental 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch_fundamental_k" -o run -- python3 "$R/bench.py" --workload fundamental --steps 1 --warmup 1 --no-cpu-baseline --no-secondary
