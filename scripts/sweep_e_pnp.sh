#!/bin/bash
# Screen the essential sweep shape (MCV_E_VARIANT: 0 = <4 models, 2 points per lane> default,
# 1 = <4,1>, 2 = <6,1>, 3 = <2,2>, 4 = <6,2>, 5 = <8,1>) and the PnP poses per wave (MCV_PNP_K).
mkdir -p gpurun_out
for v in ${EVARIANTS:-0 1 2 3 4 5}; do
    MCV_E_VARIANT=$v timeout -k 10 200 python bench.py --workload essential --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/evar_$v.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/evar_$v.log; exit $rc; }
    python -c "import json; d=json.loads([l for l in open('gpurun_out/evar_$v.log') if l.startswith('{')][0]); print('evariant $v', round(d['value']/1e6,3), 'Mhyp/s verify', round(d['kernels']['mcv_e_verify']['avg_launch_ms'],2), 'ms', d['result']['best_count'])"
done
for k in ${PNPK:-2 4 6 8}; do
    MCV_PNP_K=$k timeout -k 10 200 python bench.py --workload pnp --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pnpk_$k.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/pnpk_$k.log; exit $rc; }
    python -c "import json; d=json.loads([l for l in open('gpurun_out/pnpk_$k.log') if l.startswith('{')][0]); print('pnp K $k', round(d['value']/1e6,3), 'Mhyp/s verify', round(d['kernels']['mcv_pnp_verify']['avg_launch_ms'],3), 'ms', d['result']['best_count'])"
done
