# r03 v33: v32 + the device factorization's symbolic uploads on a host thread beside the schedule and relabelling (analyze hook): parity / factor / boundary / distributed tests, S10 construction phases
# on per subset chain; same ordering): parity / factor / boundary / distributed tests, then the
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/v33
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_factor.py tests/test_gpu_boundary.py tests/test_gpu_dist.py > gpurun_out/v33/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || exit $rc
CPK_TIMING=1 timeout -k 10 300 python -u tools/ptime.py > gpurun_out/v33/ptime.log 2>&1
echo "ptime rc $?"
