# per-rank share of the P = 8 split on one GPU (CPK_COMM=null), and its kernel trace
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dist
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/dist_timing.py 1:0 8:0 8:7 > gpurun_out/dist/timing.log 2>&1
rc=$?; echo "timing rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dist/trace -o p -- python3 tools/dist_timing.py 8:0 > gpurun_out/dist/trace.log 2>&1
echo "trace rc $?"
