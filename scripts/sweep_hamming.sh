#!/bin/bash
# Screen the Hamming grid on the cfg2 bench, one process per variant: MCV_HAMMING_WAVES (target waves
# over the (query-wave, train-chunk) grid), MCV_HAMMING_Q (queries per lane), MCV_HAMMING_NB (16-dword
# SGPR vectors per staged train group).
mkdir -p gpurun_out
for nb in ${NBS:-1 2}; do
for q in ${QS:-1}; do
for v in ${VARIANTS:-8192 16384}; do
    MCV_HAMMING_NB=$nb MCV_HAMMING_Q=$q MCV_HAMMING_WAVES=$v timeout -k 10 120 python bench.py --workload hamming --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ham_${nb}_${q}_$v.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/ham_${nb}_${q}_$v.log; exit $rc; }
    python -c "import json; d=json.loads([l for l in open('gpurun_out/ham_${nb}_${q}_$v.log') if l.startswith('{')][0]); print('NB $nb Q $q waves $v', round(d['value']/1e6,2), 'Mq/s', round(d['roofline']['avg_launch_ms']*1e3,1), 'us', round(d['roofline']['valu']['frac'],3))"
done
done
done
