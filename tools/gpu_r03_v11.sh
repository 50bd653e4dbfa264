# r03 v11: construction (Kp / Kp-in-schedule-order overlapped with the factor upload, leaner
# schedule passes, parallel Kp assembly): parity + factor tests, construction phases at S10,
# per-rank construction and iteration time at P = 8 (CPK_COMM=null)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dist
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_factor.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r03_v11_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ptime.py > gpurun_out/r03_v11_ptime.log 2>&1
rc=$?; echo "ptime rc $rc"; [ $rc -eq 0 ] || exit $rc
CPK_TIMING=1 timeout -k 10 400 python -u tools/dist_timing.py 1:0 8:0 > gpurun_out/dist/timing_v11.log 2>&1
echo "dist rc $?"
