#!/bin/bash
# L2 with the lean GEMM form as the default: matcher tests, bench line, kernel stats, PMC traffic / MFMA, rank shares.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "$R/gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -1 "$R/gpurun_out/$name.log" | cut -c1-160
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step m_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_matchers.py tests/test_gpu_pipeline.py
(
cd /tmp && export TMPDIR=/tmp
w=l2
step prof_$w 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$w" -o run -- \
    python3 "$R/bench.py" --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
step pmc_fetch_$w 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch_$w" -o run -- \
    python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
step pmc_write_$w 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write_$w" -o run -- \
    python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
step pmc_mfma_$w 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d "$R/gpurun_out/pmc_mfma_$w" -o run -- \
    python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
) || exit 1
step collect 120 python3 scripts/collect_profiles.py r04
step bench_l2 300 python bench.py --workload l2 --steps 5 --warmup 2
MCV_DIST_BACKEND=gloo step selflaunch_l2 300 python bench.py --workload l2 --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline
step l2_share 200 python scripts/exp/l2_shard_timing.py
