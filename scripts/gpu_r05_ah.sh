#!/bin/bash
# Round 5: F verify counts staged per block (one contiguous store): parity, bench, PMC write pass.
source scripts/gpu_step.sh
step test_f 600 python -u -m pytest tests/test_gpu_fundamental.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread
step bench_fundamental 300 python bench.py --workload fundamental --steps 5 --warmup 1 --cpu-seconds 8
cd /tmp && export TMPDIR=/tmp
w=fundamental
step pmc_write_$w 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write_$w" -o run -- \
    python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
step prof_$w 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$w" -o run -- \
    python3 "$R/bench.py" --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
