#!/bin/bash
# Variant screen of the certified PnP sweep: poses per wave (MCV_PNP_K) x waves per EU (MCV_PNP_WPE);
# prints the verify kernel's average launch time per variant. PARTS=t also runs the PnP GPU tests first.
set -u
mkdir -p gpurun_out/pnpsweep
export PYTHONUNBUFFERED=1
if [[ ${PARTS:-} == *t* ]]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_pnp.py -m gpu -x -q --timeout 300 --timeout-method thread \
      > gpurun_out/pnpsweep/pytest.log 2>&1 || { tail -30 gpurun_out/pnpsweep/pytest.log; exit 1; }
  tail -1 gpurun_out/pnpsweep/pytest.log
fi
# VARIANTS: space-separated K_WPE tokens
for v in ${VARIANTS:-2_3 2_4 2_5 4_3 4_4}; do
  set -- ${v/_/ }
  timeout -k 10 300 env MCV_PNP_K=$1 MCV_PNP_WPE=$2 python bench.py --workload pnp --steps 5 --warmup 2 --no-cpu-baseline \
      > gpurun_out/pnpsweep/k$1_w$2.log 2>&1 || { tail -5 gpurun_out/pnpsweep/k$1_w$2.log; exit 1; }
  python - gpurun_out/pnpsweep/k$1_w$2.log K=$1 WPE=$2 <<'PY'
import json,sys
d=json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print(sys.argv[2], sys.argv[3], "verify_ms %.3f step_ms %.3f  %.2f M hyp/s" % (d['kernels']['mcv_pnp_verify']['avg_launch_ms'], d['ms_per_step'], d['value']/1e6))
PY
done
