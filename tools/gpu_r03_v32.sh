# r03 v32: dissection without shared label / stamp counters (thread label blocks, stamps counted
# on per subset chain; same ordering): parity / factor / boundary / distributed tests, then the
# S10 construction phases (CPK_TIMING)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/v32
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_factor.py tests/test_gpu_boundary.py tests/test_gpu_dist.py > gpurun_out/v32/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || exit $rc
CPK_TIMING=1 timeout -k 10 300 python -u tools/ptime.py > gpurun_out/v32/ptime.log 2>&1
echo "ptime rc $?"
