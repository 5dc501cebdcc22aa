#!/bin/bash
# Round-2 EPnP screen: PnP GPU parity tests, then the pnp bench per solver kind.
set -o pipefail
mkdir -p gpurun_out/r02p
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_pnp.py \
    > gpurun_out/r02p/pytest_pnp.log 2>&1 || exit 2
for k in EPNP AP3P; do
  timeout -k 10 200 python bench.py --workload pnp --pnp-kind $k --steps 5 --warmup 1 --no-cpu-baseline \
      > gpurun_out/r02p/bench_pnp_$k.json 2> gpurun_out/r02p/bench_pnp_$k.err || exit 3
done
