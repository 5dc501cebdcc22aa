#!/bin/bash
# Certified PnP sweep: GPU parity (PnP tests), then the PnP bench line per poses-per-wave variant and
# against the all-fp64 sweep (MCV_PNP_FP64=1). Stops at the first failing GPU step.
set -u
R=$PWD
mkdir -p gpurun_out/pnpcert
export PYTHONUNBUFFERED=1
step() {   # name timeout cmd...
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "$R/gpurun_out/pnpcert/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -2 "$R/gpurun_out/pnpcert/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step pytest_pnp 600 python -u -m pytest tests/test_gpu_pnp.py -m gpu -x -q --timeout 300 --timeout-method thread
step bench_fp64 300 env MCV_PNP_FP64=1 python bench.py --workload pnp --steps 5 --warmup 2 --no-cpu-baseline
for k in 4 2 6 8; do
step bench_k$k 300 env MCV_PNP_K=$k python bench.py --workload pnp --steps 5 --warmup 2 --no-cpu-baseline
done
step bench_ap3p 300 python bench.py --workload pnp --pnp-kind AP3P --steps 5 --warmup 2 --no-cpu-baseline
