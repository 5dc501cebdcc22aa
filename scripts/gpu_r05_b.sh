#!/bin/bash
# Round 5: the whole GPU suite + smoke + the bench lines after the knob strip.
source scripts/gpu_step.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread
grep -h "sample:" gpurun_out/pytest_gpu.log | cut -c1-160
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_homography 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
step bench_fundamental 300 python bench.py --workload fundamental --steps 5 --warmup 1 --no-cpu-baseline
step bench_essential 300 python bench.py --workload essential --steps 5 --warmup 2 --no-cpu-baseline
step bench_pnp 300 python bench.py --workload pnp --steps 5 --warmup 2 --no-cpu-baseline
step bench_pnp_ap3p 300 python bench.py --workload pnp --pnp-kind AP3P --steps 5 --warmup 2 --no-cpu-baseline
step bench_hamming 300 python bench.py --workload hamming --steps 20 --warmup 3 --no-cpu-baseline
step bench_l2 300 python bench.py --workload l2 --steps 5 --warmup 2 --no-cpu-baseline
for f in gpurun_out/bench_*.log; do python - "$f" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")]
if l:
    d = json.loads(l[-1]); print(sys.argv[1], round(d["value"] / 1e6, 3), "M", d["ms_per_step"], d.get("result"))
PY
done
