#!/bin/bash
# Round 5 screen (experiment builds): mcv_l2_prep16's wave-trips in flight x rows per block:
# base 2 x 16, 1 = 4 x 32, 2 = 4 x 64, 3 = 2 x 64, 4 = 8 x 128 (kernel times at the full and 8-rank share).
source scripts/gpu_step.sh
MINICV_NATIVE_LIB=$R/libs/exp/2/libMiniCVNative.so step test_v2 300 python -u -m pytest tests/test_gpu_matchers.py -x -q -k l2 --timeout 120 --timeout-method thread
cd /tmp && export TMPDIR=/tmp
for v in base 1 2 3 4; do
  if [ $v != base ]; then export MINICV_NATIVE_LIB=$R/libs/exp/$v/libMiniCVNative.so; fi
  for n in 1 8; do
    step prof_pp_${v}_$n 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_pp_${v}_$n" -o run -- \
        python3 "$R/scripts/exp/l2_share_prof.py" $n
  done
done
