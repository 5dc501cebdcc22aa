#!/bin/bash
# Screen fundamental-matrix sweep shapes (MCV_F_VARIANT) on the cfg4 bench; one process per variant.
mkdir -p gpurun_out
for v in ${VARIANTS:-0 1 2 3 4 5 6 7}; do
    MCV_F_VARIANT=$v timeout -k 10 200 python bench.py --workload fundamental --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/fvariant_$v.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/fvariant_$v.log; exit $rc; }
    python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/fvariant_$v.log') if l.startswith('{')][0]); print('fvariant $v', round(d['value']/1e6,3), 'Mhyp/s', round(d['roofline']['avg_launch_ms'],2), 'ms', d['result']['best_count'])"
done
