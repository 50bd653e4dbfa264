# r03 v28 (re-entry validation): full GPU suite at HEAD, construction phases with the layout
# sub-phases (CPK_TIMING), S10 bench with its PMC passes and CPU baseline
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/v28
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread --durations=25 > gpurun_out/v28/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || exit $rc
CPK_TIMING=1 timeout -k 10 300 python -u tools/ptime.py > gpurun_out/v28/ptime.log 2>&1
rc=$?; echo "ptime rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/v28/bench_s10.json 2> gpurun_out/v28/bench_s10.err
echo "bench rc $?"
