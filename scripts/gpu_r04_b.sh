#!/bin/bash
# Round 4 screens: PnP two-tier prefilter vs the exact-only bound, Hamming GEMM vs popcount form,
# L2 f16 form with 1 or 2 query sets per wave (correctness of the QT=2 kernel first).
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {   # name timeout cmd...
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "$R/gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; grep -h '^{' "$R/gpurun_out/$name.log" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d.get('roofline',{}); k=d.get('kernels',{})
    print('  value %.4g ms/step %.3f kernel %s %.4f ms frac %.3f' % (d['value'], d['ms_per_step'], r.get('kernel'), r.get('avg_launch_ms') or 0, r.get('frac') or 0))
" 2>/dev/null; tail -1 "$R/gpurun_out/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
PARTS=${PARTS:-tphl}
if [[ $PARTS == *t* ]]; then
MCV_L2_QT=2 step test_l2_qt2 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_matchers.py -k l2
fi
if [[ $PARTS == *p* ]]; then
step pnp_tiers2 300 python bench.py --workload pnp --steps 3 --warmup 1 --no-cpu-baseline
MCV_PNP_TIERS=1 step pnp_tiers1 300 python bench.py --workload pnp --steps 3 --warmup 1 --no-cpu-baseline
step pnp_tiers2b 300 python bench.py --workload pnp --steps 3 --warmup 1 --no-cpu-baseline
fi
if [[ $PARTS == *h* ]]; then
step ham_gemm 300 python bench.py --workload hamming --steps 20 --warmup 3 --no-cpu-baseline
MCV_HAMMING_FORM=popcount step ham_popcount 300 python bench.py --workload hamming --steps 20 --warmup 3 --no-cpu-baseline
fi
if [[ $PARTS == *l* ]]; then
step l2_qt1 300 python bench.py --workload l2 --steps 5 --warmup 2 --no-cpu-baseline
MCV_L2_QT=2 step l2_qt2 300 python bench.py --workload l2 --steps 5 --warmup 2 --no-cpu-baseline
fi
