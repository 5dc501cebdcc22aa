#!/bin/bash
# Round 5 screen: the f16-domain exact scan with the next tile's fragments loaded under the current
# tile's filter vs HEAD; kernel times by rocprofv3 at the full and the 8-rank share.
source scripts/gpu_step.sh
step test_match 300 python -u -m pytest tests/test_gpu_matchers.py -x -q --timeout 120 --timeout-method thread
cd /tmp && export TMPDIR=/tmp
for v in new old; do
  if [ $v = old ]; then export MINICV_NATIVE_LIB=$R/libs/old/libMiniCVNative.so; fi
  for n in 1 8; do
    step prof_${v}_$n 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_scan_${v}_$n" -o run -- \
        python3 "$R/scripts/exp/l2_share_prof.py" $n
  done
done
