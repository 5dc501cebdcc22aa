#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r02d
for v in 2 20 21 22 23; do
  MCV_HCERT_NOREDO=1 MCV_HCERT_VARIANT=$v timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline \
      > gpurun_out/r02d/bench_h_v$v.json 2> gpurun_out/r02d/bench_h_v$v.err || exit 3
done
