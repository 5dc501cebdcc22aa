#!/bin/bash
# One-piece split generate: the homography parity tests, then the headline bench line three times.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_homography.py tests/test_gpu_multishard.py tests/test_gpu_pipeline.py tests/test_gpu_plan_guard.py > gpurun_out/pytest.log 2>&1 || { tail -30 gpurun_out/pytest.log; exit 1; }
tail -2 gpurun_out/pytest.log
for rep in 1 2 3; do
  timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/h_$rep.json 2>gpurun_out/h.err || { tail -5 gpurun_out/h.err; exit 1; }
  python3 -c "import json;j=json.load(open('gpurun_out/h_$rep.json'));print($rep, round(j['value']/1e6,2), round(j['ms_per_step'],3), j['kernels'], j.get('result'))"
done
