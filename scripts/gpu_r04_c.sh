#!/bin/bash
# Hamming GEMM-form variants (query tiles per wave, accumulator double buffer), correctness first.
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
step() {   # name timeout cmd...
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "$R/gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; summ "$R/gpurun_out/$name.log"; tail -1 "$R/gpurun_out/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step test_ham 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_matchers.py -k hamming
MCV_HAMMING_QT=1 step test_ham_qt1 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_matchers.py -k hamming
MCV_HAMMING_DB=0 step test_ham_db0 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_matchers.py -k hamming
for v in "2 1" "2 0" "1 1" "1 0"; do set -- $v
    MCV_HAMMING_QT=$1 MCV_HAMMING_DB=$2 step ham_qt$1_db$2 300 python bench.py --workload hamming --steps 50 --warmup 5 --no-cpu-baseline
done
for w in 2048 8192; do
    MCV_HAMMING_WAVES=$w step ham_w$w 300 python bench.py --workload hamming --steps 50 --warmup 5 --no-cpu-baseline
done
