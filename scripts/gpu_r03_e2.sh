#!/bin/bash
# Round 3: F sweep over point chunks (MCV_F_WAVES screen), E / F sweep shapes after the linear Sampson cut,
# PnP at K = 3; parity of F / E / PnP.
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
step tests 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_fundamental.py tests/test_gpu_essential.py tests/test_gpu_pnp.py tests/test_gpu_multishard.py
for w in 0 16384 65536 262144; do
    step bench_f_w$w 300 env MCV_F_WAVES=$w python bench.py --workload fundamental --steps 10 --warmup 3 --no-cpu-baseline --no-secondary
done
for pk in 4 2 1 3; do
    step bench_f_pk$pk 300 env MCV_F_PK=$pk python bench.py --workload fundamental --steps 10 --warmup 3 --no-cpu-baseline --no-secondary
done
for pk in 0 1 2 3; do
    step bench_e_pk$pk 300 env MCV_E_PK=$pk python bench.py --workload essential --steps 5 --warmup 2 --no-cpu-baseline
done
for c in 0 16384 50000; do
    step bench_e_c$c 300 env MCV_E_CHUNK=$c python bench.py --workload essential --steps 5 --warmup 2 --no-cpu-baseline
done
step bench_pnp 300 python bench.py --workload pnp --steps 5 --warmup 2 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
for w in fundamental essential; do
    step sq2_$w 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
        --output-format csv -d "$R/gpurun_out/sq2_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-secondary
done
