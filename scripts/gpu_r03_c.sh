#!/bin/bash
# Round 3: element-major (bank-conflict-free) eigen workspace of the H / F generate kernels — parity under
# MCV_EIG_SOA=1, then the cfg3 / cfg4 benches with both layouts, and the LDS counters of each.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {   # name timeout cmd...
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "$R/gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -3 "$R/gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step tests_soa 600 env MCV_EIG_SOA=1 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_homography.py tests/test_gpu_fundamental.py -k "bit_exact or stress or full_size or cfg or golden or vs_oracle"
step tests_e 300 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_essential.py -k edge
for soa in 0 1; do
    step bench_h_soa$soa 300 env MCV_EIG_SOA=$soa python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary
    step bench_f_soa$soa 300 env MCV_EIG_SOA=$soa python bench.py --workload fundamental --steps 10 --warmup 3 --no-cpu-baseline --no-secondary
done
cd /tmp && export TMPDIR=/tmp
for soa in 0 1; do
    step lds_soa$soa 120 env MCV_EIG_SOA=$soa rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
        --output-format csv -d "$R/gpurun_out/lds_soa$soa" -o run -- \
        python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-secondary
done
