#!/bin/bash
# Round-6 refresh after the one-piece H generate: the full GPU suite, smoke, the homography bench lines,
# their rocprofv3 kernel stats and the generate's SQ pass (the other workloads' evidence is unchanged).
source scripts/gpu_step.sh
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_homography 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 8
step bench_homography_fused 300 python bench.py --steps 10 --warmup 3 --fused --no-cpu-baseline
step bench_homography_fast 300 python bench.py --steps 10 --warmup 3 --fast-minimal --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
step prof_homography 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_homography" -o run -- \
    python3 "$R/bench.py" --workload homography --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
step pmc_gen_h 120 rocprofv3 --kernel-trace --kernel-include-regex "mcv_h_gen" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY \
    --output-format csv -d "$R/gpurun_out/pmc_gen_h" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-secondary
