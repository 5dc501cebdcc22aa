#!/bin/bash
# E solvePoly split from the model phase (mcv_e5_solve<WAVES>): tests + kernel times per waves-per-SIMD.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for w in 2 4; do
    MCV_E5_SOLVE_WAVES=$w timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_essential.py > gpurun_out/e5w_tests$w.log 2>&1
    rc=$?; tail -1 gpurun_out/e5w_tests$w.log; [ $rc -ne 0 ] && exit $rc
done
cd /tmp && export TMPDIR=/tmp
for v in 1 2 3 4; do
    MCV_E5_SOLVE_WAVES=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_e5s$v" -o run -- \
        python3 "$R/bench.py" --workload essential --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > "$R/gpurun_out/e5s$v.log" 2>&1 || exit 1
    python3 -c "
import csv,glob
f=glob.glob('$R/gpurun_out/prof_e5s$v/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'e5_' in r['Name']: print('w$v', r['Name'][:40], r['Calls'], '%.3f ms'%(float(r['AverageNs'])/1e6))
"
done
