#!/bin/bash
# L2 GEMM: default (per-tile min-test epilogue) vs s_setprio 1 around the MFMA cluster (form 5), alternating.
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
for f in 0 5 0 5; do
    MCV_L2_FORM=$f step l2g_$f 300 python bench.py --workload l2 --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
done
MCV_L2_FORM=5 step l2f5_tests 600 python -u -m pytest tests -m gpu -x -q -k "l2 or L2" --timeout 300 --timeout-method thread
