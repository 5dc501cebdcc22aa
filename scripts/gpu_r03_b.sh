#!/bin/bash
# Round 3: E parity after the branch-free Durand-Kerner sweep, E / AP3P benches, SQ counter passes of the
# PnP / F / E sweeps (issue fractions from measured instruction counts) and the PnP sweep's writes.
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
step tests 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_essential.py tests/test_gpu_selftest.py
step bench_e 300 python bench.py --workload essential --steps 5 --warmup 2 --no-cpu-baseline
step bench_e_fast 300 python bench.py --workload essential --steps 5 --warmup 2 --no-cpu-baseline --fast-minimal
step bench_ap3p 300 python bench.py --workload pnp --pnp-kind AP3P --steps 5 --warmup 2 --no-cpu-baseline
step bench_ap3p_fast 300 python bench.py --workload pnp --pnp-kind AP3P --steps 5 --warmup 2 --no-cpu-baseline --fast-minimal
cd /tmp && export TMPDIR=/tmp
step prof_e 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_e" -o run -- \
    python3 "$R/bench.py" --workload essential --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
for w in pnp fundamental essential; do
    step sq_$w 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
        --output-format csv -d "$R/gpurun_out/sq_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-secondary
done
step wr_pnp 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/wr_pnp" -o run -- \
    python3 "$R/bench.py" --workload pnp --steps 2 --warmup 1 --no-cpu-baseline --no-secondary
