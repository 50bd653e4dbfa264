# r03 v2: parity of the lane-owned level loop, then A/B of the level loop variants
# (base: owned rows without per-level barriers; own1: owned rows with barriers; own0: the
# previous loop), and per-XCD round-0 stamps
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_factor.py -x -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/r03_v2_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_ab.sh own1 own0 || exit $?
timeout -k 10 300 env CPK_LIB_PATH=$GRAFT_REPO_ROOT/abv/stamps/libcpk.so python -u tools/pipe_stamps.py > gpurun_out/r03_v2_stamps.log 2>&1
echo "stamps rc $?"
