#!/bin/bash
# Screen the L2 MFMA matcher's train rows per tile (MCV_L2_TR: 32 = one MFMA chain per wave, 64 = two) on the cfg5 bench.
mkdir -p gpurun_out
for v in ${VARIANTS:-32 64}; do
    MCV_L2_TR=$v timeout -k 10 120 python bench.py --workload l2 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/l2_$v.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/l2_$v.log; exit $rc; }
    python -c "import json; d=json.loads([l for l in open('gpurun_out/l2_$v.log') if l.startswith('{')][0]); print('TR $v', round(d['value'],1), 'TF/s', round(d['roofline']['avg_launch_ms'],3), 'ms', round(d['roofline']['frac'],3))"
done
