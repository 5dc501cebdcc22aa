#!/bin/bash
# Pipelined H evaluate (MCV_H_PIPE pieces: generate of piece j+1 beside the sweep of piece j): tests + step times.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
MCV_H_PIPE=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_homography.py > gpurun_out/pipe_tests.log 2>&1
rc=$?; tail -2 gpurun_out/pipe_tests.log; [ $rc -ne 0 ] && exit $rc
for v in 1 2 4 8 16; do
    MCV_H_PIPE=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/pipe_$v.log 2>&1 || exit 1
    echo "== pipe $v"; grep -h '^{' gpurun_out/pipe_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('  value %.4g ms/step %.3f verify %.3f gen %.3f' % (d['value'], d['ms_per_step'], d['kernels']['verify'], d['kernels']['generate']))"
done
