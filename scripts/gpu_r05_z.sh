#!/bin/bash
# Round 5 refresh after the stream-K partitions of the L2 and Hamming GEMMs: matcher parity, their bench
# lines, kernel-trace stats, PMC traffic / MFMA passes and the rank-share timings (L2 share).
source scripts/gpu_step.sh
step test_match 300 python -u -m pytest tests/test_gpu_matchers.py -x -q --timeout 120 --timeout-method thread
step bench_hamming 300 python bench.py --workload hamming --steps 50 --warmup 5
step bench_l2 300 python bench.py --workload l2 --steps 10 --warmup 2
step rank_share 600 python scripts/exp/rank_share_timing.py
cd /tmp && export TMPDIR=/tmp
for w in hamming l2; do
    step prof_$w 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
    step pmc_fetch_$w 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
    step pmc_write_$w 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
    step pmc_mfma_$w 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE \
        --output-format csv -d "$R/gpurun_out/pmc_mfma_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
done
