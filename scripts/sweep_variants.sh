#!/bin/bash
# Screen sweep shapes (MCV_SWEEP_VARIANT) on the headline bench; one process per variant.
mkdir -p gpurun_out
for v in ${VARIANTS:-0 1 2 3 4 5 0}; do
    MCV_SWEEP_VARIANT=$v timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/variant_$v.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/variant_$v.log; exit $rc; }
    python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/variant_$v.log') if l.startswith('{')][0]); print('variant $v', round(d['value']/1e6,2), 'Mhyp/s', round(d['roofline']['avg_launch_ms'],2), 'ms', d['result']['best_count'])"
done
