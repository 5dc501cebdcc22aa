#!/bin/bash
# Round-6 iteration: the steps named in $STEPS (space-separated) of the list below, each under its own
# time limit, stopping at the first failure (scripts/gpu_step.sh).
source scripts/gpu_step.sh
PT="python -u -m pytest -m gpu -x -q -rA --timeout 300 --timeout-method thread"
for st in ${STEPS:-}; do
case $st in
  t_ham) step t_ham 600 $PT tests/test_gpu_matchers.py tests/test_gpu_matcher_shards.py tests/test_gpu_pipeline.py -k "hamming or Hamming or multi or pipeline or match_features" ;;
  t_match) step t_match 900 $PT tests/test_gpu_matchers.py tests/test_gpu_matcher_shards.py tests/test_gpu_pipeline.py ;;
  t_e) step t_e 900 $PT tests/test_gpu_essential.py ;;
  t_h) step t_h 900 $PT tests/test_gpu_homography.py tests/test_gpu_multishard.py tests/test_gpu_plan_guard.py tests/test_gpu_pipeline.py tests/test_gpu_selftest.py ;;
  t_f) step t_f 900 $PT tests/test_gpu_fundamental.py ;;
  t_pnp) step t_pnp 900 $PT tests/test_gpu_pnp.py ;;
  t_all) step t_all 1100 $PT tests ;;
  b_ham) step b_ham 300 python bench.py --workload hamming --steps 200 --warmup 10 ;;
  b_l2) step b_l2 300 python bench.py --workload l2 --steps 20 --warmup 3 ;;
  b_h) step b_h 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 8 ;;
  b_e) step b_e 300 python bench.py --workload essential --steps 5 --warmup 2 --no-cpu-baseline ;;
  b_f) step b_f 300 python bench.py --workload fundamental --steps 5 --warmup 1 --no-cpu-baseline ;;
  b_pnp) step b_pnp 300 python bench.py --workload pnp --steps 5 --warmup 2 --no-cpu-baseline ;;
  rank_share) step rank_share 600 python scripts/exp/rank_share_timing.py ;;
  p_*) w=${st#p_}; (cd /tmp && export TMPDIR=/tmp && step prof_$w 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$w" -o run -- python3 "$R/bench.py" --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-secondary) || exit 1 ;;
  w_*) w=${st#w_}; (cd /tmp && export TMPDIR=/tmp && step pmc_write_$w 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write_$w" -o run -- python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary) || exit 1 ;;
  m_*) w=${st#m_}; (cd /tmp && export TMPDIR=/tmp && step pmc_mfma_$w 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/pmc_mfma_$w" -o run -- python3 "$R/bench.py" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary) || exit 1 ;;
  *) echo "unknown step $st"; exit 3 ;;
esac
done
