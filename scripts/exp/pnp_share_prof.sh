set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for h in 131072 262144; do
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pnp_$h -o run -- python3 $R/bench.py --workload pnp --hyps $h --steps 6 --warmup 2 --no-cpu-baseline --no-secondary > $R/gpurun_out/pnp_$h.json 2> $R/gpurun_out/pnp_$h.err || exit 1
done
echo ok
