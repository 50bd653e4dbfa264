# r03 v41: one rank's share at P = 8 (CPK_COMM=null) with the new default sweep configuration
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/v41
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/dist_timing.py 8:0 > gpurun_out/v41/dist_timing.log 2>&1
echo "dist rc $?"
