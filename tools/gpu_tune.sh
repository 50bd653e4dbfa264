set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
C="192,576,64,2048,8192,512 192,576,64,1024,4096,256 192,576,64,1024,4096,512 192,576,64,512,2048,256 192,576,64,512,2048,512 192,576,64,2048,8192,1024 192,576,64,1024,4096,1024"
N=1250000 timeout -k 10 900 python tools/tune_sweep.py $C > gpurun_out/tune_small.log 2>&1
N=10000000 timeout -k 10 900 python tools/tune_sweep.py $C > gpurun_out/tune.log 2>&1
