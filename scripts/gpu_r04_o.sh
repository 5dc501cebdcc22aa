#!/bin/bash
# L2 GEMM form screen: MCV_L2_QT = 1 (default) / 3 (two query sets per wave, one accumulator set); exactness + time.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
MCV_L2_QT=5 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matchers.py -k "l2" > gpurun_out/qt3_tests.log 2>&1
rc=$?; tail -2 gpurun_out/qt3_tests.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for v in 1 5 6 1 5; do
    MCV_L2_QT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_qt$v" -o run -- \
        python3 "$R/bench.py" --workload l2 --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/qt$v.log" 2>&1 || exit 1
    echo "== qt $v"; grep -h '^{' "$R/gpurun_out/qt$v.log" | cut -c1-120
    python3 -c "
import csv,glob
f=glob.glob('$R/gpurun_out/prof_qt$v/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'mfma' in r['Name']: print(r['Name'][:40], r['Calls'], '%.3f ms'%(float(r['AverageNs'])/1e6))
"
done
