# round-3 end: the driver's GPU suite command (timed, with --durations) and the default bench line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
s=$(date +%s)
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 600 --timeout-method thread --durations=40 > gpurun_out/r03_full_pytest.log 2>&1
rc=$?; echo "pytest rc $rc wall $(( $(date +%s) - s )) s"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 240 python bench.py > gpurun_out/r03_full_bench.json 2> gpurun_out/r03_full_bench.err
echo "bench rc $?"
