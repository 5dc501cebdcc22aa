#!/bin/bash
# Screen sweep shapes (MCV_SWEEP_VARIANT) on the headline bench; one process per variant.
#   0 / 20-30: packed-f32 sweep mcv_h_verify_pk<K, pairs per lane> (0 = <8, 2>; 27-30 = <5,2> <7,2> <6,3> <6,2>;
#   after the running-min change: 0 = <6,2> 29.45, <5,2> 29.80, <7,2> 29.44, <6,3> 29.39, <8,2> 28.89 ms,
#   so <8,2> became the default); 19: scalar mcv_h_verify<6, 2>.
mkdir -p gpurun_out
for v in ${VARIANTS:-0 19 20 21 22 24 25 26}; do
    MCV_SWEEP_VARIANT=$v timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/variant_$v.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/variant_$v.log; exit $rc; }
    python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/variant_$v.log') if l.startswith('{')][0]); print('variant $v', round(d['value']/1e6,2), 'Mhyp/s', round(d['roofline']['avg_launch_ms'],2), 'ms', d['result']['best_count'])"
done
