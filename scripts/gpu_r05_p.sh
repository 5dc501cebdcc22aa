#!/bin/bash
# Round 5 checkpoint: the whole -m gpu suite, smoke, and every bench workload at N=1.
source scripts/gpu_step.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_homography 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 8
step bench_fundamental 300 python bench.py --workload fundamental --steps 5 --warmup 1 --cpu-seconds 8
step bench_essential 300 python bench.py --workload essential --steps 5 --warmup 2 --cpu-seconds 8
step bench_pnp 300 python bench.py --workload pnp --steps 5 --warmup 2 --cpu-seconds 8
step bench_pnp_ap3p 300 python bench.py --workload pnp --pnp-kind AP3P --steps 5 --warmup 2 --cpu-seconds 8
step bench_hamming 300 python bench.py --workload hamming --steps 50 --warmup 5
step bench_l2 300 python bench.py --workload l2 --steps 10 --warmup 2
step bench_scaled 300 python bench.py --workload scaled --steps 5 --warmup 2 --cpu-seconds 8
