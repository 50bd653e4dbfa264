# r03 v26: one rank's share at P = 8 (CPK_COMM=null) after the fused cpminres update, under a few
# round-0 / upper staging configurations (smaller round-0 blocks pipeline more blocks per workgroup)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dist
export TMPDIR=/tmp
CPK_SWEEPS=";128,384,64;96,288,64;256,768,64;192,576,64,512,2048,256" timeout -k 10 600 python -u tools/dist_timing.py 8:0 > gpurun_out/dist/timing_v26.log 2>&1
echo "dist rc $?"
