#!/bin/bash
# SQ counter passes of the L2 f16-split kernel (MFMA busy, VALU / LDS instruction counts, waits).
set -u
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
run() {
    local name=$1; shift
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$R/gpurun_out/$name" -o run -- \
        python3 "$R/bench.py" --workload l2 --steps 2 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/$name.log" 2>&1
    local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run l2pmc_a SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE
run l2pmc_b SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SALU
