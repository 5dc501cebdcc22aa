#!/bin/bash
# After the L2 epilogue change: the full GPU suite + smoke, the L2 bench line, its kernel-trace, traffic
# and MFMA passes, and the L2 rank-share timings.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {   # name timeout cmd...
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "$R/gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -2 "$R/gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_l2 300 python bench.py --workload l2 --steps 5 --warmup 2
MCV_DIST_BACKEND=gloo step selflaunch_l2 300 python bench.py --workload l2 --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline
step l2_share 200 python scripts/exp/l2_shard_timing.py
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
