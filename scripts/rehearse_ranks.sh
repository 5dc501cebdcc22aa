#!/bin/bash
# Rehearse bench.py's multi-rank path on a one-GPU box: 2 ranks share the device and the single
# all-reduce goes through gloo (MCV_DIST_BACKEND=gloo). A correctness check of the sharding and
# the global-best exchange, not a measurement (the driver runs N ranks on N GPUs over RCCL).
set -u
mkdir -p gpurun_out
export MCV_DIST_BACKEND=gloo
port=29611
for w in ${WORKLOADS:-homography fundamental essential pnp hamming l2 scaled}; do
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port $port bench.py --workload $w --gpus 2 --steps 2 --warmup 1 \
        --no-cpu-baseline > gpurun_out/rehearse_$w.log 2>&1
    rc=$?
    echo "$w rc=$rc"
    [ $rc -ne 0 ] && { tail -5 gpurun_out/rehearse_$w.log; exit $rc; }
    grep -h '^{' gpurun_out/rehearse_$w.log | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(' ', d['n_gpus'], d['value'], d.get('result'))"
    port=$((port + 1))
done
