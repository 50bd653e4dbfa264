# r03 v27: one rank's share at P = 8 (CPK_COMM=null) with the fused cpminres update, and without it
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dist
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/dist_timing.py 8:0 > gpurun_out/dist/timing_v27.log 2>&1
rc=$?; echo "dist rc $rc"; [ $rc -eq 0 ] || exit $rc
CPK_NO_MINRES_FUSE=1 timeout -k 10 300 python -u tools/dist_timing.py 8:0 > gpurun_out/dist/timing_v27_nofuse.log 2>&1
echo "dist nofuse rc $?"
