#!/bin/bash
# PnP: EPnP generate of piece j + 1 beside the sweep of piece j (MCV_PNP_PIPE = pieces, default 8) vs
# one generate then one sweep (MCV_PNP_PIPE=0), alternating; then the PnP GPU tests under the default.
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
    d=json.loads(l); print(d['ms_per_step'], d['roofline'].get('avg_launch_ms'), d['roofline'].get('launches'), d['value'])" || true
    if [ $rc -ne 0 ]; then tail -15 "$R/gpurun_out/$name.log"; exit $rc; fi
}
step pnp_tests 600 python -u -m pytest tests/test_gpu_pnp.py -x -q -m gpu --timeout 300 --timeout-method thread
for v in 8 0 4 16 8 0; do
    MCV_PNP_PIPE=$v step pipe_$v 300 python bench.py --workload pnp --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
done
MCV_PNP_PIPE=8 step pipe_ap3p 300 python bench.py --workload pnp --pnp-kind AP3P --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
