#!/bin/bash
# Round 3: XCD-aware chunk order of the F / E sweeps (MCV_XCD_MAP A/B) with FETCH_SIZE, parity of F / E.
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
step tests 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_fundamental.py tests/test_gpu_essential.py tests/test_gpu_multishard.py
for x in 0 1; do
    step bench_f_x$x 300 env MCV_XCD_MAP=$x python bench.py --workload fundamental --steps 10 --warmup 3 --no-cpu-baseline --no-secondary
    step bench_e_x$x 300 env MCV_XCD_MAP=$x python bench.py --workload essential --steps 5 --warmup 2 --no-cpu-baseline
done
cd /tmp && export TMPDIR=/tmp
for x in 0 1; do
    step fetch_f_x$x 120 env MCV_XCD_MAP=$x rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/fetch_f_x$x" -o run -- \
        python3 "$R/bench.py" --workload fundamental --steps 2 --warmup 1 --no-cpu-baseline --no-secondary
done
