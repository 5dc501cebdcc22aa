#!/bin/bash
# Iteration helper: a chosen subset of GPU tests (-k expression in $TESTS, test files in $FILES),
# bench lines ($BENCHES: "name|args" entries separated by ';') and a kernel-trace profile of the
# first bench ($PROF=1). Stops at the first failing GPU step.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {   # name timeout cmd...
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "$R/gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -3 "$R/gpurun_out/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
if [ -n "${FILES:-}" ]; then
    step pytest_iter 600 python -u -m pytest $FILES -m gpu -x -q -rf --timeout 120 --timeout-method thread ${TESTS:+-k "$TESTS"}
fi
IFS=';' read -ra BL <<< "${BENCHES:-}"
for b in "${BL[@]}"; do
    [ -z "$b" ] && continue
    name=${b%%|*}; args=${b#*|}
    step bench_$name 300 python bench.py $args
done
if [ "${PROF:-0}" = 1 ] && [ ${#BL[@]} -gt 0 ]; then
    b=${BL[0]}; name=${b%%|*}; args=${b#*|}
    cd /tmp && export TMPDIR=/tmp
    step prof_$name 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$name" -o run -- \
        python3 "$R/bench.py" $args --no-cpu-baseline
fi
