#!/bin/bash
# Round 5: sampled matcher timing; SQ counters of the EPnP generate.
source scripts/gpu_step.sh
step tests_g 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_matchers.py tests/test_gpu_selftest.py
step bench_hamming 300 python bench.py --workload hamming --steps 50 --warmup 5 --no-cpu-baseline
step bench_l2 300 python bench.py --workload l2 --steps 10 --warmup 2 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
step pmc_gen_pnp 120 timeout -s KILL 100 rocprofv3 --kernel-trace --kernel-include-regex "pnp_generate" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU \
    --output-format csv -d "$R/gpurun_out/pmc_gen_pnp" -o run -- python3 "$R/bench.py" --workload pnp --steps 2 --warmup 1 --no-cpu-baseline --no-secondary
