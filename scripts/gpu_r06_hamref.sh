#!/bin/bash
# Round-6 refresh after the fp4 Hamming GEMM: the matcher GPU tests, the Hamming bench line, per-size
# timings, rocprofv3 kernel stats and the PMC passes for the Hamming workload.
source scripts/gpu_step.sh
step pytest_gpu_match 600 python -u -m pytest tests/test_gpu_matchers.py tests/test_gpu_matcher_shards.py tests/test_gpu_pipeline.py -m gpu -x -q -rA --timeout 300 --timeout-method thread
step bench_hamming 300 python bench.py --workload hamming --steps 50 --warmup 5
step ham_sizes 300 python -u scripts/exp/ham_size_timing.py
cd /tmp && export TMPDIR=/tmp
step prof_hamming 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_hamming" -o run -- \
    python3 "$R/bench.py" --workload hamming --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
step pmc_fetch_hamming 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch_hamming" -o run -- \
    python3 "$R/bench.py" --workload hamming --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
step pmc_write_hamming 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write_hamming" -o run -- \
    python3 "$R/bench.py" --workload hamming --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
step pmc_mfma_hamming 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d "$R/gpurun_out/pmc_mfma_hamming" -o run -- \
    python3 "$R/bench.py" --workload hamming --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
