#!/bin/bash
# Certified H sweep shape re-screen at the round-3 code: default <6,1> vs its VOPC-e32 form (7) and <5,1> (8).
set -o pipefail
mkdir -p gpurun_out/r03s
export PYTHONUNBUFFERED=1
for v in 0 7 8 0 7; do
  MCV_HCERT_VARIANT=$v timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline \
      > gpurun_out/r03s/bench_h_v$v.json 2> gpurun_out/r03s/bench_h_v$v.err || exit 3
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r03s/bench_h_v$v.json').read().strip().splitlines()[-1]); print('v$v', d['kernels'])"
done
