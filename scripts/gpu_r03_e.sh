set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_tests.sh tests/test_gpu_essential.py tests/test_gpu_cv_sampler.py || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_e -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload essential --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > $GRAFT_REPO_ROOT/gpurun_out/bench_e.log 2>&1
