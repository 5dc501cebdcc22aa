#!/bin/bash
# Round 5: PnP verify full trips from the pair layout (no bounds / address selects): parity, bench, SQ pass.
source scripts/gpu_step.sh
step tests_l 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pnp.py
step bench_pnp 300 python bench.py --workload pnp --steps 5 --warmup 2 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
step prof_pnp 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_pnp_l" -o run --output-format csv -- python3 "$R/bench.py" --workload pnp --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
step pmc_sq_pnp 120 timeout -s KILL 100 rocprofv3 --kernel-trace --kernel-include-regex "pnp_verify|epnp_split" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d "$R/gpurun_out/pmc_sq_pnp_l" -o run -- python3 "$R/bench.py" --workload pnp --steps 1 --warmup 1 --no-cpu-baseline --no-secondary
step pmc_sqv_pnp 120 timeout -s KILL 100 rocprofv3 --kernel-trace --kernel-include-regex "pnp_verify|epnp_split" --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 --output-format csv -d "$R/gpurun_out/pmc_sqv_pnp_l" -o run -- python3 "$R/bench.py" --workload pnp --steps 1 --warmup 1 --no-cpu-baseline --no-secondary
