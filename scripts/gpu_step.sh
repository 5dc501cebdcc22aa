#!/bin/bash
# Helper sourced by the round-5 GPU scripts: step NAME TIMEOUT CMD... runs CMD under its own time limit,
# logs to gpurun_out/NAME.log, prints the tail and stops the script at the first failure.
set -u
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {
    local name=$1 tmo=$2; shift 2
    timeout -k 10 "$tmo" "$@" > "$R/gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -3 "$R/gpurun_out/$name.log" | cut -c1-400
    if [ $rc -ne 0 ]; then exit $rc; fi
}
