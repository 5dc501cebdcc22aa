#!/bin/bash
# SQ counters of the Hamming GEMM kernel (one rocprofv3 --pmc pass per counter set).
set -u
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d "$R/gpurun_out/pmc_ham_sq" -o run -- python3 "$R/bench.py" --workload hamming --steps 5 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/pmc_ham_sq.log" 2>&1
echo "rc=$?"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SALU \
    --output-format csv -d "$R/gpurun_out/pmc_ham_sq2" -o run -- python3 "$R/bench.py" --workload hamming --steps 5 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/pmc_ham_sq2.log" 2>&1
echo "rc=$?"
