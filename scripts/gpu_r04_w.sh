#!/bin/bash
# PnP verify: lane-granular recount log (default) vs the trip recount (MCV_PNP_LANE=0): the PnP tests,
# then the PnP bench both ways and a kernel-trace of the default.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "$R/gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; grep -h '^{' "$R/gpurun_out/$name.log" | cut -c1-260 || true
    if [ $rc -ne 0 ]; then tail -15 "$R/gpurun_out/$name.log"; exit $rc; fi
}
step pnp_tests 600 python -u -m pytest tests/test_gpu_pnp.py -x -q -m gpu --timeout 300 --timeout-method thread
step bench_pnp_lane 300 python bench.py --workload pnp --steps 3 --warmup 1 --no-cpu-baseline
MCV_PNP_LANE=0 step bench_pnp_trip 300 python bench.py --workload pnp --steps 3 --warmup 1 --no-cpu-baseline
step bench_pnp_lane2 300 python bench.py --workload pnp --steps 3 --warmup 1 --no-cpu-baseline
(
cd /tmp && export TMPDIR=/tmp
step prof_pnp_lane 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_pnp_lane" -o run -- \
    python3 "$R/bench.py" --workload pnp --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
) || exit 1
