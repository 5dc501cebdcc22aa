#!/bin/bash
# Round 5 screen: EPnP betas / pose kernels at one vs two waves per EU.
source scripts/gpu_step.sh
step tests_s 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pnp.py -k "epnp or EPNP or full or counts"
MCV_EXP_WPE2=1 step tests_s2 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pnp.py -k "epnp or EPNP or full or counts"
cd /tmp && export TMPDIR=/tmp
step prof_w1 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_pnp_w1" -o run --output-format csv -- python3 "$R/bench.py" --workload pnp --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
MCV_EXP_WPE2=1 step prof_w2 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_pnp_w2" -o run --output-format csv -- python3 "$R/bench.py" --workload pnp --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
