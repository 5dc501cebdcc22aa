#!/bin/bash
# Round 5: stall breakdown of the matcher GEMMs (wave-parked / issue-stall / active, LDS stalls and
# bank conflicts, MFMA busy) — one SQ pass per workload.
source scripts/gpu_step.sh
cd /tmp && export TMPDIR=/tmp
for w in hamming l2; do
step pmc_stall_$w 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
    --output-format csv -d "$R/gpurun_out/pmc_stall_$w" -o run -- \
    python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
done
