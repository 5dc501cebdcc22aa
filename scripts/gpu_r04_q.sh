#!/bin/bash
# L2 rank shares: the chunk-count model vs fixed 15 / 11 chunks (scripts/exp/l2_shard_timing.py per variant), twice.
set -u
mkdir -p gpurun_out
for v in "model 0" "c15 15" "c11 11" "model 0" "c15 15"; do
    set -- $v
    MCV_L2_CHUNKS=$2 timeout -k 10 120 python3 scripts/exp/l2_shard_timing.py > gpurun_out/l2c_$1.log 2>&1 || exit 1
    echo "$1 $(grep -h '^{' gpurun_out/l2c_$1.log | python3 -c "import sys,json; print(' '.join('%d:%.3f' % (d['ranks'], d['ms']) for d in map(json.loads, sys.stdin)))")"
done
