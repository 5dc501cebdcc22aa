#!/bin/bash
# Hamming GEMM form v3 (keys in the accumulator, in-register expansion): tests, bench, SQ counters.
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
MCV_HAMMING_SUB=1 step test_ham_sub1 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_matchers.py -k hamming
for sub in 2 1; do
  for w in 4096 8192 16384; do
    MCV_HAMMING_SUB=$sub MCV_HAMMING_WAVES=$w step ham_s${sub}_w$w 300 python bench.py --workload hamming --steps 50 --warmup 5 --no-cpu-baseline
  done
done
[[ ${PMC:-1} == 0 ]] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d "$R/gpurun_out/pmc_ham3_sq" -o run -- python3 "$R/bench.py" --workload hamming --steps 5 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/pmc_ham3_sq.log" 2>&1
echo "pmc rc=$?"
