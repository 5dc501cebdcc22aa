# Screen (needs a build whose PnP verify launcher reads MCV_SCREEN; the product ignores it): the
# resident-wave tail chunking (1) or 2 / 4 poses per wave (2 / 4) against the default (0), at the 8-rank share and 2^20.
for rep in 1 2; do for v in ${VARIANTS:-0 1}; do for h in 131072 1048576; do
  MCV_SCREEN=$v timeout -k 10 120 python bench.py --workload pnp --hyps $h --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/pt_${v}_${h}.log 2>&1 || exit 1
  python3 -c "import json,sys; l=[x for x in open('gpurun_out/pt_${v}_${h}.log') if x.startswith('{')][-1]; j=json.loads(l); print('v=$v h=$h ms', round(j['ms_per_step'],3), 'verify', j.get('roofline',{}).get('avg_launch_ms'))"
done; done; done
