#!/bin/bash
# Round 5: EPnP generate with row-register Jacobi sweeps; Hamming with packet-timed launches.
source scripts/gpu_step.sh
step tests_f 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pnp.py tests/test_gpu_matchers.py
step bench_pnp 300 python bench.py --workload pnp --steps 5 --warmup 2 --no-cpu-baseline
step bench_hamming 300 python bench.py --workload hamming --steps 50 --warmup 5 --no-cpu-baseline
step ham_gap 200 python scripts/exp/ham_gap.py 200
cat gpurun_out/ham_gap.log
cd /tmp && export TMPDIR=/tmp
step prof_pnp 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_pnp" -o run -- python3 "$R/bench.py" --workload pnp --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
