#!/bin/bash
# F / E sweeps: the lane log of undecided (point, model) lanes (default) vs the in-loop re-test
# (MCV_SPK_LOG=0), alternating; then the F / E GPU tests under the default.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "$R/gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; grep -h '^{' "$R/gpurun_out/$name.log" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['ms_per_step'], d['roofline'].get('avg_launch_ms'), d['value'])" || true
    if [ $rc -ne 0 ]; then tail -15 "$R/gpurun_out/$name.log"; exit $rc; fi
}
step fe_tests 900 python -u -m pytest tests/test_gpu_fundamental.py tests/test_gpu_essential.py -x -q -m gpu --timeout 300 --timeout-method thread
for v in 1 0 1 0; do
    MCV_SPK_LOG=$v step f_log$v 300 python bench.py --workload fundamental --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
done
for v in 1 0 1 0; do
    MCV_SPK_LOG=$v step e_log$v 300 python bench.py --workload essential --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
done
