#!/bin/bash
# Round 3: sample search and solve apart in the hypothesis functions (one solve pass per wave) — the
# H / F / E / PnP benches, both eigen workspace layouts, the PnP verify K screen, parity of the touched paths.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {   # name timeout cmd...
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "$R/gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -2 "$R/gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
for soa in 0 1; do
    step bench_h_soa$soa 300 env MCV_EIG_SOA=$soa python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary
    step bench_f_soa$soa 300 env MCV_EIG_SOA=$soa python bench.py --workload fundamental --steps 10 --warmup 3 --no-cpu-baseline --no-secondary
done
step bench_e 300 python bench.py --workload essential --steps 5 --warmup 2 --no-cpu-baseline
step bench_e_fast 300 python bench.py --workload essential --steps 5 --warmup 2 --no-cpu-baseline --fast-minimal
for k in 3 4 5; do
    step bench_pnp_k$k 300 env MCV_PNP_K=$k python bench.py --workload pnp --steps 5 --warmup 2 --no-cpu-baseline
done
step bench_ap3p 300 python bench.py --workload pnp --pnp-kind AP3P --steps 5 --warmup 2 --no-cpu-baseline
step tests 900 python -u -m pytest -v -rA --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_homography.py tests/test_gpu_fundamental.py tests/test_gpu_essential.py tests/test_gpu_pnp.py \
    tests/test_gpu_cv_sampler.py tests/test_gpu_multishard.py
