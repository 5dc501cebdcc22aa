#!/bin/bash
# Round 5: L2 launch fusion (5 launches, no empty kernels) + lane-parallel F/E count writes +
# pooled profiling events: matcher / F / E tests, L2 share timing, Hamming step anatomy, benches,
# kernel traces of the L2 shares and F / E write counters.
source scripts/gpu_step.sh
step tests_c 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_matchers.py tests/test_gpu_pipeline.py tests/test_gpu_fundamental.py tests/test_gpu_essential.py
step l2_share 200 python scripts/exp/l2_shard_timing.py
cat gpurun_out/l2_share.log
step ham_gap 200 python scripts/exp/ham_gap.py 200
cat gpurun_out/ham_gap.log
step bench_l2 300 python bench.py --workload l2 --steps 10 --warmup 2 --no-cpu-baseline
step bench_hamming 300 python bench.py --workload hamming --steps 50 --warmup 5 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
step prof_l2share 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_l2share" -o run -- python3 "$R/scripts/exp/l2_shard_timing.py"
step prof_ham 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_ham" -o run -- python3 "$R/scripts/exp/ham_gap.py" 50
step pmc_write_fundamental 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write_fundamental" -o run -- \
    python3 "$R/bench.py" --workload fundamental --steps 2 --warmup 1 --no-cpu-baseline --no-secondary
step pmc_write_essential 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write_essential" -o run -- \
    python3 "$R/bench.py" --workload essential --steps 2 --warmup 1 --no-cpu-baseline --no-secondary
cd "$R"
step bench_fundamental 300 python bench.py --workload fundamental --steps 5 --warmup 1 --no-cpu-baseline
step bench_essential 300 python bench.py --workload essential --steps 5 --warmup 2 --no-cpu-baseline
