#!/bin/bash
# Round 4, multi-GPU readiness on the one-GPU box:
#  1. bench.py --gpus 2 launches its own ranks (no torch.distributed.run); MCV_DIST_BACKEND=gloo lets
#     the two ranks share the device. Every workload must print one line with n_gpus 2.
#  2. what one rank computes at N = 1 / 2 / 4 / 8 (scripts/exp/rank_share_timing.py).
#  3. the cfg4 line at 2^20 hypotheses.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {   # name timeout cmd...
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "$R/gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -2 "$R/gpurun_out/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
PARTS=${PARTS:-tplsb}
if [[ $PARTS == *t* ]]; then
step pytest_guard 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_plan_guard.py tests/test_gpu_cv_sampler.py tests/test_gpu_fundamental.py tests/test_gpu_essential.py tests/test_gpu_matchers.py tests/test_gpu_pnp.py}
fi
if [[ $PARTS == *l* ]]; then
for w in ${WORKLOADS:-homography fundamental essential pnp hamming l2 scaled}; do
    MCV_DIST_BACKEND=gloo step selflaunch_$w 300 python bench.py --workload $w --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline
done
fi
if [[ $PARTS == *s* ]]; then
step rank_share 600 python scripts/exp/rank_share_timing.py
fi
if [[ $PARTS == *b* ]]; then
step bench_fundamental 300 python bench.py --workload fundamental --steps 5 --warmup 1 --cpu-seconds 8
fi
if [[ $PARTS == *p* ]]; then
step bench_pnp 300 python bench.py --workload pnp --steps 5 --warmup 2 --no-cpu-baseline
step bench_pnp_ap3p 300 python bench.py --workload pnp --pnp-kind AP3P --steps 5 --warmup 2 --no-cpu-baseline
fi
