# r03 v19: the refinement turn (sptrsv_turn_kernel: backward round 0 of the first solve, the
# residual and forward round 0 of the refinement solve in one pass): parity (parity + factor
# files, the S10 headline test), then S10 A/B against no_turn
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_factor.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r03_v19_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -x -q -m gpu --timeout 240 --timeout-method thread -k "s10_one_gpu" > gpurun_out/r03_v19_scale.log 2>&1
rc=$?; echo "scale rc $rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab2.sh base noturn:CPK_NO_TURN=1 base2 noturn2:CPK_NO_TURN=1 || exit $?
