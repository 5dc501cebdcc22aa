#!/bin/bash
# findScaled with group-ahead observation staging: tests, bench line, kernel stats.
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
step s_tests 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_scaled.py
(
cd /tmp && export TMPDIR=/tmp
step prof_scaled 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_scaled" -o run -- \
    python3 "$R/bench.py" --workload scaled --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
) || exit 1
step bench_scaled 300 python bench.py --workload scaled --steps 5 --warmup 2 --cpu-seconds 8
