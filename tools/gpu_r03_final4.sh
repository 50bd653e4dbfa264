# r03 final4: the new default sweep configuration -- full GPU suite, S10 bench (PMC + CPU baseline), rocprofv3 kernel stats
# kernel stats of the same bench command, S10 construction phases
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final4
export TMPDIR=/tmp
timeout -k 10 840 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread --durations=15 > gpurun_out/final4/pytest_gpu.log 2>&1
echo "pytest ok"
timeout -k 10 600 python bench.py > gpurun_out/final4/bench_s10.json 2> gpurun_out/final4/bench_s10.err
echo "bench ok"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final4/prof -o bench -- python3 bench.py --steps 5 --no-cpu-baseline --no-pmc > gpurun_out/final4/prof_bench.json 2> gpurun_out/final4/prof_bench.err
echo "rocprof ok"
