#!/bin/bash
# One-piece EPnP generate: the PnP parity tests, the PnP bench line and the PnP rank shares.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pnp.py tests/test_gpu_multishard.py > gpurun_out/pytest.log 2>&1 || { tail -30 gpurun_out/pytest.log; exit 1; }
tail -1 gpurun_out/pytest.log
timeout -k 10 300 python -u bench.py --workload pnp --steps 5 --warmup 2 --cpu-seconds 8 > gpurun_out/bench_pnp.log 2>&1 || { tail -5 gpurun_out/bench_pnp.log; exit 1; }
tail -1 gpurun_out/bench_pnp.log | cut -c1-200
timeout -k 10 300 python -u bench.py --workload pnp --pnp-kind AP3P --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_pnp_ap3p.log 2>&1 || { tail -5 gpurun_out/bench_pnp_ap3p.log; exit 1; }
timeout -k 10 600 python -u scripts/exp/rank_share_timing.py pnp > gpurun_out/share.jsonl 2>&1 || { tail -5 gpurun_out/share.jsonl; exit 1; }
tail -1 gpurun_out/share.jsonl
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_pnp" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload pnp --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > "$GRAFT_REPO_ROOT/gpurun_out/prof_pnp.log" 2>&1
