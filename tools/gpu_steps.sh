#!/bin/bash
# One parameterised GPU call: bash tools/gpu_steps.sh <tag> <step> [<step> ...]
# Output under gpurun_out/<tag>/, one file per step (step index in the name).  Every step runs
# under its own time limit; the first failing step ends the call (no GPU work after a fault).
#
# Steps (quote a step that carries arguments: 'bench=--steps 5 --no-pmc'):
#   tests[=<pytest args>]     pytest -m gpu (default: the whole GPU suite)
#   smoke                     __graft_entry__.smoke()
#   bench[=<bench args>]      the bench.py line (JSON)
#   rocprof[=<bench args>]    rocprofv3 --kernel-trace --stats of the same bench.py command
#   pmc=<counters>[@<args>]   one rocprofv3 --pmc pass (<= 8 SQ, 4 TCC counters) over bench.py --pmc-probe <args>
#   dist[=<P:r ...>]          tools/dist_timing.py (one rank's share of a P-way solve)
#   distprof[=<P:r ...>]      rocprofv3 kernel trace of tools/dist_timing.py
#   py=<script> [args]        python -u <script> [args]
#   sh=<command>              any other command (bash -c)
# Limits: tests 900 s, bench / rocprof / pmc / py 600 s, others 300 s.
tag=$1
shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for step in "$@"; do
    i=$((i + 1))
    name=${step%%=*}
    arg=""
    [ "$name" != "$step" ] && arg=${step#*=}
    f="$out/$(printf %02d $i)_$name"
    echo "[$(date +%T)] step $i: $step"
    case $name in
    tests)
        timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread --durations=15 \
            ${arg} > "$f.log" 2>&1 ;;
    smoke)
        timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > "$f.log" 2>&1 ;;
    bench)
        timeout -k 10 600 python -u bench.py ${arg} > "$f.json" 2> "$f.err" ;;
    rocprof)
        timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$f" -o bench -- \
            python3 bench.py ${arg} > "$f.json" 2> "$f.err" ;;
    pmc)
        ctr=${arg%%@*}
        pa=""
        [ "$ctr" != "$arg" ] && pa=${arg#*@}
        timeout -s KILL 300 rocprofv3 --pmc ${ctr} --output-format csv -d "$f" -o pmc -- \
            python3 bench.py --pmc-probe ${pa} > "$f.json" 2> "$f.err" ;;
    dist)
        timeout -k 10 300 python -u tools/dist_timing.py ${arg} > "$f.log" 2>&1 ;;
    distprof)
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$f" -o dist -- \
            python3 tools/dist_timing.py ${arg} > "$f.log" 2>&1 ;;
    py)
        timeout -k 10 600 python -u ${arg} > "$f.log" 2>&1 ;;
    sh)
        timeout -k 10 600 bash -c "${arg}" > "$f.log" 2>&1 ;;
    *)
        echo "unknown step $name"; exit 2 ;;
    esac
    rc=$?
    echo "[$(date +%T)] step $i: rc $rc"
    if [ $rc -ne 0 ]; then
        tail -20 "$f".* 2>/dev/null
        exit $rc
    fi
done
