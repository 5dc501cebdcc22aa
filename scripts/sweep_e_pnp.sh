#!/bin/bash
# Screen the essential path's shapes and the PnP poses per wave:
#   MCV_E_PK     packed-prefilter sweep: 0 = <3 pairs, 2 points per lane> (default), 1 = <2,2>,
#                2 = <4,1>, 3 = <2,1>, 9 = the fp64 sweep (then MCV_E_VARIANT picks its shape)
#   MCV_E_ROOTS  split-path root finder: 4 = 4-lane groups (default), 8, 1 = one lane
#   MCV_PNP_K    PnP poses per wave (2 / 4 / 6 / 8)
mkdir -p gpurun_out
show() {   # log label
    python -c "import json; d=json.loads([l for l in open('$1') if l.startswith('{')][0]); k=d['kernels']; print('$2', round(d['value']/1e6,3), 'Mhyp/s', {n: round(v['avg_launch_ms'],3) for n, v in k.items()}, d['result']['best_count'])"
}
for v in ${EPK:-0 1 2 3 9}; do
    MCV_E_PK=$v timeout -k 10 200 python bench.py --workload essential --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/epk_$v.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/epk_$v.log; exit $rc; }
    show gpurun_out/epk_$v.log "E_PK $v"
done
for v in ${EROOTS:-4 8 1}; do
    MCV_E_ROOTS=$v timeout -k 10 200 python bench.py --workload essential --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/eroots_$v.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/eroots_$v.log; exit $rc; }
    show gpurun_out/eroots_$v.log "E_ROOTS $v"
done
for k in ${PNPK:-2 4 6 8}; do
    MCV_PNP_K=$k timeout -k 10 200 python bench.py --workload pnp --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pnpk_$k.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/pnpk_$k.log; exit $rc; }
    show gpurun_out/pnpk_$k.log "PNP_K $k"
done
