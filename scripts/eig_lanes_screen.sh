#!/bin/bash
# Screen lanes per block of the eigen (JacobiImpl_) H hypothesis kernel (MCV_EIG_LANES).
set -u
mkdir -p gpurun_out
for L in 39 40 39 40; do
    MCV_EIG_LANES=$L timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/el_$L.log 2>&1 || exit 1
    echo -n "L=$L "; python -c "
import json; l=[x for x in open('gpurun_out/el_$L.log') if x.startswith('{')][0]; d=json.loads(l); print(round(d['value']/1e6,2), d['kernels']['generate'])"
done
