# r03 v30: construction with insertion-sorted layout rows, threaded layout zero-fills, the parallel Schur graph and reserved dissection vectors (same ordering, factor and layout): parity / factor / boundary tests, then the S10 construction phases (CPK_TIMING, with the dissection top levels)
# histograms (same factor, schedule and layout): parity / factor / distributed tests, then the
# S10 construction phases (CPK_TIMING)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/v30
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_factor.py tests/test_gpu_boundary.py > gpurun_out/v30/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || exit $rc
CPK_TIMING=1 timeout -k 10 300 python -u tools/ptime.py > gpurun_out/v30/ptime.log 2>&1
echo "ptime rc $?"
