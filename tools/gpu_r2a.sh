# round 2: full GPU suite, then the headline-size parity tests
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_factor.py -x -v --timeout 120 --timeout-method thread > gpurun_out/factor.log 2>&1
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --deselect tests/test_gpu_scale.py --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py -x -v -s --timeout 900 --timeout-method thread > gpurun_out/scale.log 2>&1
