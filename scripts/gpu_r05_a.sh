#!/bin/bash
# Round 5: full-range parity samples of the F / E / PnP bench workloads, then the GPU suite.
source scripts/gpu_step.sh
step range_tests 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_fundamental.py::test_full_size_cfg4 tests/test_gpu_essential.py::test_e_counts_bench_workload_full \
    tests/test_gpu_pnp.py::test_pnp_counts_bench_workload_full
grep -h "sample:" gpurun_out/range_tests.log | cut -c1-200
