#!/bin/bash
# Screens: PnP poses per wave with the exact-tier sweep; L2 per-rank kernel breakdown at the 8-rank share.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
summ() { grep -h '^{' "$1" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d.get('roofline',{})
    print('  value %.4g ms/step %.4f kernel %s %.4f ms frac %.3f' % (d['value'], d['ms_per_step'], r.get('kernel'), r.get('avg_launch_ms') or 0, r.get('frac') or 0))
" 2>/dev/null; }
step() {
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "$R/gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; summ "$R/gpurun_out/$name.log"; tail -1 "$R/gpurun_out/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
for k in 2 3 4; do
    MCV_PNP_K=$k step pnp_k$k 300 python bench.py --workload pnp --steps 3 --warmup 1 --no-cpu-baseline --hyps 262144
done
cd /tmp && export TMPDIR=/tmp
step prof_l2share 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_l2share" -o run -- \
    python3 "$R/scripts/exp/l2_shard_timing.py"
cat "$R/gpurun_out/prof_l2share/run_kernel_stats.csv" | head -20
