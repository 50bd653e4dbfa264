# r03 v1: the GPU suite without the headline-size file (durations), the S10 bench with the
# cost-balanced round-0 assignment and with the stride (r0_stride), and the round-0 tail stamps
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests -x -q -m "gpu and not slow" --timeout 300 --timeout-method thread --durations=40 > gpurun_out/r03_v1_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; ok $rc || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/r03_v1_bench.json 2> gpurun_out/r03_v1_bench.err
rc=$?; echo "bench rc $rc"; [ $rc -eq 0 ] || exit $rc
CPK_R0_STRIDE=1 timeout -k 10 600 python bench.py --no-cpu-baseline --no-pmc > gpurun_out/r03_v1_bench_stride.json 2> gpurun_out/r03_v1_bench_stride.err
rc=$?; echo "bench stride rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 env CPK_LIB_PATH=$GRAFT_REPO_ROOT/abv/stamps/libcpk.so python -u tools/pipe_stamps.py > gpurun_out/r03_v1_stamps.log 2>&1
echo "stamps rc $?"
