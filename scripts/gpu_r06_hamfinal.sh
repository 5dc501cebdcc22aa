#!/bin/bash
# Round-6 closing run after the fp4 Hamming GEMM: the full GPU suite, smoke, the Hamming bench line.
source scripts/gpu_step.sh
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_hamming 300 python bench.py --workload hamming --steps 50 --warmup 5
