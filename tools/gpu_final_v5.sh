# r02 v5 validation: S10 bench (PMC + CPU baseline), rocprof kernel stats of the same command,
# the GPU suite without the headline-size file, smoke, then the S10 headline-size parity test
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python bench.py > gpurun_out/bench_s10.json 2> gpurun_out/bench_s10.err
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 5 --no-cpu-baseline --no-pmc > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
timeout -k 10 540 python -u -m pytest tests -x -q -m gpu --deselect tests/test_gpu_scale.py --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
