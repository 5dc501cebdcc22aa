#!/bin/bash
# Round 5: L2 GEMM with the per-XCD stream-K partition.
source scripts/gpu_step.sh
step tests_w 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_matchers.py
step bench_l2 300 python bench.py --workload l2 --steps 10 --warmup 2 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
step prof_w 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_l2_w" -o run --output-format csv -- python3 "$R/bench.py" --workload l2 --steps 5 --warmup 1 --no-cpu-baseline --no-secondary
cd "$R"
step l2_share 300 python scripts/exp/l2_shard_timing.py
