# round 2: full GPU suite, bench, then the headline-size parity tests
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --deselect tests/test_gpu_scale.py --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_s10.json 2> gpurun_out/bench_s10.err
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py -x -v -s --timeout 900 --timeout-method thread > gpurun_out/scale.log 2>&1
