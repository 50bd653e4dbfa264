# r03 v7: distributed payloads packed by the sweeps' write-back (separator exchange, Kp halo):
# the distributed GPU tests, then one rank's share of P = 8 and its kernel trace
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dist
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_boundary.py -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/r03_v7_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u tools/dist_timing.py 1:0 8:0 8:3 > gpurun_out/dist/timing_v7.log 2>&1
rc=$?; echo "timing rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dist/trace_v7 -o p -- python3 tools/dist_timing.py 8:0 > gpurun_out/dist/trace_v7.log 2>&1
echo "trace rc $?"
