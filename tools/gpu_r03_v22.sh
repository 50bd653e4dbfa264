# r03 v22 (v23: residual inside the prefix kernel): the distributed refinement residual without the Kp halo exchange (Precond::tkr): the
# distributed test file (SimComm P = 2, 3, 4, 8), then one rank's share at P = 8 (CPK_COMM=null)
# with and without it
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dist
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r03_v23_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/dist_timing.py 8:0 8:3 > gpurun_out/dist/timing_v23.log 2>&1
rc=$?; echo "dist rc $rc"; [ $rc -eq 0 ] || exit $rc
CPK_NO_TKR=1 timeout -k 10 400 python -u tools/dist_timing.py 8:0 8:3 > gpurun_out/dist/timing_v23_notkr.log 2>&1
echo "dist notkr rc $?"
