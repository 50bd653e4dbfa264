#!/bin/bash
# Steps in order, each a full shell command under its own time limit, stopping at the first
# failure (no GPU work after a fault or a timeout): bash tools/gpu_run.sh <tag> "<limit>:<name>:<command>" ...
# Output of step <name> in gpurun_out/<tag>/<name>.log.
tag=$1
shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for spec in "$@"; do
    lim=${spec%%:*}
    rest=${spec#*:}
    name=${rest%%:*}
    cmd=${rest#*:}
    echo "[$(date +%T)] $name: $cmd"
    timeout -k 10 "$lim" bash -c "$cmd" > "$out/$name.log" 2>&1
    rc=$?
    echo "[$(date +%T)] $name: rc $rc"
    if [ $rc -ne 0 ]; then
        tail -25 "$out/$name.log"
        exit $rc
    fi
done
