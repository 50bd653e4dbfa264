set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k sweep > gpurun_out/pytest_sweep.log 2>&1
C="192,576,64,1024,4096,512 192,576,32,1024,4096,512 128,384,32,1024,4096,512 256,768,32,1024,4096,512"
N=10000000 timeout -k 10 900 python tools/tune_sweep.py $C > gpurun_out/tune.log 2>&1
N=1250000 timeout -k 10 900 python tools/tune_sweep.py $C > gpurun_out/tune_small.log 2>&1
