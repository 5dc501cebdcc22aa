#!/bin/bash
# PnP finalize with fewer host round trips: parity tests, the bench line and the rank shares.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pnp.py tests/test_gpu_multishard.py > gpurun_out/pytest.log 2>&1 || { tail -30 gpurun_out/pytest.log; exit 1; }
tail -2 gpurun_out/pytest.log
timeout -k 10 600 python -u scripts/exp/rank_share_timing.py pnp > gpurun_out/share.jsonl 2>&1 || { tail -5 gpurun_out/share.jsonl; exit 1; }
cat gpurun_out/share.jsonl
