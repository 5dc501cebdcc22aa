#!/bin/bash
# Self-launch rehearsal of the default (weak-scaling homography) workload at 2 and 4 ranks sharing the
# one device through gloo, plus the closing scaled bench / kernel stats on the final code.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "$R/gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; grep -h '^{' "$R/gpurun_out/$name.log" | cut -c1-200 || true
    if [ $rc -ne 0 ]; then tail -5 "$R/gpurun_out/$name.log"; exit $rc; fi
}
MCV_DIST_BACKEND=gloo step selflaunch_homography2 300 python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline
MCV_DIST_BACKEND=gloo step selflaunch_homography4 400 python bench.py --gpus 4 --steps 2 --warmup 1 --no-cpu-baseline
MCV_DIST_BACKEND=gloo step selflaunch_pnp2 300 python bench.py --workload pnp --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline
(
cd /tmp && export TMPDIR=/tmp
step prof_scaled 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_scaled" -o run -- \
    python3 "$R/bench.py" --workload scaled --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
) || exit 1
step bench_scaled 300 python bench.py --workload scaled --steps 5 --warmup 2 --cpu-seconds 8
