# r03 v34: one rank's share at P = 8 (CPK_COMM=null) after the construction speedups: per-rank
# construction phases (CPK_TIMING) and the iteration time
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/v34
export TMPDIR=/tmp
CPK_TIMING=1 timeout -k 10 300 python -u tools/dist_timing.py 8:0 > gpurun_out/v34/dist_timing.log 2>&1
echo "dist rc $?"
