# r03 final (third session): full GPU suite, S10 bench (PMC passes + CPU baseline), rocprofv3
# kernel stats of the same bench command, S10 construction phases
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final3
export TMPDIR=/tmp
timeout -k 10 840 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread --durations=15 > gpurun_out/final3/pytest_gpu.log 2>&1
echo "pytest ok"
timeout -k 10 600 python bench.py > gpurun_out/final3/bench_s10.json 2> gpurun_out/final3/bench_s10.err
echo "bench ok"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final3/prof -o bench -- python3 bench.py --steps 5 --no-cpu-baseline --no-pmc > gpurun_out/final3/prof_bench.json 2> gpurun_out/final3/prof_bench.err
echo "rocprof ok"
