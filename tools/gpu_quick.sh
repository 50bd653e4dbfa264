set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_factor.py -x -q --timeout 120 --timeout-method thread > gpurun_out/p21.log 2>&1
timeout -k 10 300 python -u tools/tune_sweep.py 192,576,64,1024,4096,512 > gpurun_out/tune.log 2>&1
CPK_NO_COL16=1 timeout -k 10 300 python -u tools/tune_sweep.py 192,576,64,1024,4096,512 >> gpurun_out/tune.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/b21.json 2> gpurun_out/b21.err
