# r03 v31: v30 + the device factorization's symbolic uploads on a host thread beside the layout, insertion-sorted relabel columns: parity / factor / boundary tests, S10 construction phases
# histograms (same factor, schedule and layout): parity / factor / distributed tests, then the
# S10 construction phases (CPK_TIMING)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/v31
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_factor.py tests/test_gpu_boundary.py > gpurun_out/v31/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || exit $rc
CPK_TIMING=1 timeout -k 10 300 python -u tools/ptime.py > gpurun_out/v31/ptime.log 2>&1
echo "ptime rc $?"
