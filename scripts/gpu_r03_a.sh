#!/bin/bash
# Round 3: parity of the touched paths, then the essential / PnP benches with rocprofv3 kernel stats.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {   # name timeout cmd...
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "$R/gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -3 "$R/gpurun_out/$name.log"
    # a plain test failure (1) lets the benches run; faults, aborts and time limits end the script
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step tests 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_essential.py tests/test_gpu_cv_sampler.py tests/test_gpu_pnp.py tests/test_gpu_multishard.py \
    tests/test_gpu_homography.py tests/test_gpu_matchers.py
step bench_e 300 python bench.py --workload essential --steps 5 --warmup 2 --no-cpu-baseline
step bench_pnp 300 python bench.py --workload pnp --steps 5 --warmup 2 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
step prof_e 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_e" -o run -- \
    python3 "$R/bench.py" --workload essential --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
step prof_pnp 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_pnp" -o run -- \
    python3 "$R/bench.py" --workload pnp --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
