#!/bin/bash
# Screen lanes per block of the eigen (JacobiImpl_) hypothesis kernels: H bench generate time.
set -u
mkdir -p gpurun_out
for L in 32 39 48 64; do
    MCV_EIG_LANES=$L timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/eig_screen_$L.log 2>&1 || exit 1
    echo "L=$L"; python -c "
import json; l=[x for x in open('gpurun_out/eig_screen_$L.log') if x.startswith('{')][0]; d=json.loads(l); print(d['value']/1e6, d['kernels'])"
done
