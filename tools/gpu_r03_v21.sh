# r03 v21: forward round 2 inside round 1's launch (dependency counters, last producer runs the
# block): parity + factor files, the S10 headline test, S10 A/B against no_chain2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_factor.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r03_v21_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -x -q -m gpu --timeout 240 --timeout-method thread -k "s10_one_gpu" > gpurun_out/r03_v21_scale.log 2>&1
rc=$?; echo "scale rc $rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab2.sh base nochain:CPK_NO_CHAIN2=1 base2 nochain2:CPK_NO_CHAIN2=1 || exit $?
