# r03 v4: the GPU suite without the headline-size file (distributed device factorization and
# refactorization, plan agreement), S10 bench with refined slot speeds, stamps
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m "gpu and not slow" --timeout 300 --timeout-method thread --durations=25 > gpurun_out/r03_v4_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_ab2.sh base || exit $?
timeout -k 10 300 env CPK_LIB_PATH=$GRAFT_REPO_ROOT/abv/stamps/libcpk.so python -u tools/pipe_stamps.py > gpurun_out/r03_v4_stamps.log 2>&1
echo "stamps rc $?"
