set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 900 python tools/tune_sweep.py 256,768,128,2048,8192,256 192,576,64,2048,8192,512 256,768,64,2048,8192,256 > gpurun_out/tune.log 2>&1
CPK_NO_PIPE=1 timeout -k 10 300 python tools/tune_sweep.py 256,768,128,2048,8192,256 192,576,64,2048,8192,512 512,1536,128,2048,8192,256 >> gpurun_out/tune.log 2>&1
