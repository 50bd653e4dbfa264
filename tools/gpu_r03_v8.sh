# r03 v8: distributed packing incl. the separator solve's halo; threaded symbolic factorization:
# distributed and factor GPU tests, P = 8 per-rank timing, construction time by phase
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dist
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_factor.py tests/test_gpu_boundary.py -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/r03_v8_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u tools/dist_timing.py 1:0 8:0 8:3 > gpurun_out/dist/timing_v8.log 2>&1
rc=$?; echo "timing rc $rc"; [ $rc -eq 0 ] || exit $rc
CPK_SYMT=1 timeout -k 10 600 python -u tools/ptime.py > gpurun_out/r03_v8_ptime.log 2>&1
echo "ptime rc $?"
