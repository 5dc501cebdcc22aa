#!/bin/bash
# Round-6 evidence: full GPU suite, smoke, every bench line, --gpus 2 self-launch (gloo, one device),
# rank-share timings, rocprofv3 kernel-trace stats per workload, PMC traffic passes, SQ (VALU / MFMA)
# passes. Stops at the first failing GPU step. PARTS: any of t (tests), b (benches), p (profiles),
# c (counters); default all.
source scripts/gpu_step.sh
PARTS=${PARTS:-tbpc}
if [[ $PARTS == *t* ]]; then
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $PARTS == *b* ]]; then
step bench_homography 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 8
step bench_homography_fused 300 python bench.py --steps 10 --warmup 3 --fused --no-cpu-baseline
step bench_homography_fast 300 python bench.py --steps 10 --warmup 3 --fast-minimal --no-cpu-baseline
step bench_fundamental 300 python bench.py --workload fundamental --steps 5 --warmup 1 --cpu-seconds 8
step bench_hamming 300 python bench.py --workload hamming --steps 50 --warmup 5
step bench_l2 300 python bench.py --workload l2 --steps 10 --warmup 2
step bench_essential 300 python bench.py --workload essential --steps 5 --warmup 2 --cpu-seconds 8
step bench_pnp 300 python bench.py --workload pnp --steps 5 --warmup 2 --cpu-seconds 8
step bench_pnp_ap3p 300 python bench.py --workload pnp --pnp-kind AP3P --steps 5 --warmup 2 --no-cpu-baseline
step bench_essential_fast 300 python bench.py --workload essential --steps 5 --warmup 2 --no-cpu-baseline --fast-minimal
step bench_scaled 300 python bench.py --workload scaled --steps 5 --warmup 2 --cpu-seconds 8
for w in fundamental l2; do
    MCV_DIST_BACKEND=gloo step selflaunch_$w 300 python bench.py --workload $w --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline
done
step rank_share 600 python scripts/exp/rank_share_timing.py
fi
cd /tmp && export TMPDIR=/tmp
if [[ $PARTS == *p* ]]; then
for w in homography fundamental essential pnp hamming l2 scaled; do
    step prof_$w 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
done
fi
[[ $PARTS == *c* ]] || exit 0
for w in homography fundamental essential pnp hamming l2 scaled; do
    step pmc_fetch_$w 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
    step pmc_write_$w 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
done
for w in homography fundamental essential pnp; do
    step pmc_sq_$w 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
        --output-format csv -d "$R/gpurun_out/pmc_sq_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
done
for w in hamming l2; do
    step pmc_mfma_$w 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE \
        --output-format csv -d "$R/gpurun_out/pmc_mfma_$w" -o run -- \
        python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
done
# the split H generate's two passes (round 6)
step pmc_gen_h 120 rocprofv3 --kernel-trace --kernel-include-regex "mcv_h_gen" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY \
    --output-format csv -d "$R/gpurun_out/pmc_gen_h" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-secondary
# the PnP kernels by instruction class
step pmc_sqv_pnp 120 rocprofv3 --kernel-trace --kernel-include-regex "pnp_verify|epnp_split" --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 \
    --output-format csv -d "$R/gpurun_out/pmc_sqv_pnp" -o run -- python3 "$R/bench.py" --workload pnp --steps 1 --warmup 1 --no-cpu-baseline --no-secondary
