set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python tools/tune_sweep.py 192,576,64,2048,8192,512 > gpurun_out/tune_spmv.log 2>&1
