# kernel trace of one rank's share of a P-way solve (CPK_COMM=null timing stand-in)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/dtrace
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dtrace -o dt -- python3 tools/dist_timing.py "$@" > gpurun_out/dtrace.log 2>&1
