# r03 v3: round-0 assignment by dispatch-slot speed + lane-owned backward levels: parity subset,
# A/B against the stride, and stamps
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/r03_v3_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_ab2.sh base stride:CPK_R0_STRIDE=1 base2 || exit $?
timeout -k 10 300 env CPK_LIB_PATH=$GRAFT_REPO_ROOT/abv/stamps/libcpk.so python -u tools/pipe_stamps.py > gpurun_out/r03_v3_stamps.log 2>&1
echo "stamps rc $?"
