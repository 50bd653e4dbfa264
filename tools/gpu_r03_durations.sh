# round-3 start: per-test durations of the whole GPU suite (the driver's command plus
# --durations), the default S10 bench line, and the round-0 per-block cycles
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }  # pass, or ordinary test failures: go on
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 900 --timeout-method thread --durations=80 > gpurun_out/r03_durations.log 2>&1
rc=$?; echo "pytest rc $rc"; ok $rc || exit $rc
timeout -k 10 300 env CPK_LIB_PATH=$GRAFT_REPO_ROOT/abv/stamps/libcpk.so python -u tools/blk_cycles.py > gpurun_out/blk_cycles.log 2>&1
rc=$?; echo "blk_cycles rc $rc"; ok $rc || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r03_bench0.json 2> gpurun_out/r03_bench0.err
echo "bench rc $?"
