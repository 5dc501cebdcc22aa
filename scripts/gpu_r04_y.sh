#!/bin/bash
# PnP verify poses per wave (MCV_PNP_K) with the lane-granular recount log: 2 / 3 / 4.
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
    d=json.loads(l); print(d['ms_per_step'], d['roofline'].get('avg_launch_ms'))" || true
    if [ $rc -ne 0 ]; then tail -15 "$R/gpurun_out/$name.log"; exit $rc; fi
}
for k in 3 2 4 3; do
    MCV_PNP_K=$k step pnpk_$k 300 python bench.py --workload pnp --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
done
