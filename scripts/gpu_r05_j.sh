#!/bin/bash
# Round 5: split EPnP generate (half the SVD matrix in registers, 4 waves/CU); F/E verify counts added
# per block in LDS (one atomic per model and chunk group): parity, benches, kernel times, WRITE_SIZE.
source scripts/gpu_step.sh
step tests_j 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pnp.py tests/test_gpu_fundamental.py tests/test_gpu_essential.py
step bench_pnp 300 python bench.py --workload pnp --steps 5 --warmup 2 --no-cpu-baseline
step bench_fundamental 300 python bench.py --workload fundamental --steps 3 --warmup 1 --no-cpu-baseline
step bench_essential 300 python bench.py --workload essential --steps 3 --warmup 1 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
step prof_pnp 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_pnp_j" -o run --output-format csv -- python3 "$R/bench.py" --workload pnp --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
step pmc_write_fundamental 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write_fundamental_j" -o run -- python3 "$R/bench.py" --workload fundamental --steps 1 --warmup 1 --no-cpu-baseline --no-secondary
step pmc_write_essential 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write_essential_j" -o run -- python3 "$R/bench.py" --workload essential --steps 1 --warmup 1 --no-cpu-baseline --no-secondary
