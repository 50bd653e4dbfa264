set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 600 python bench.py --size 1250000 --no-cpu-baseline --no-pmc > gpurun_out/bench_small.json 2> gpurun_out/bench_small.err
timeout -k 10 600 python bench.py --no-cpu-baseline --no-pmc > gpurun_out/bench_s10q.json 2> gpurun_out/bench_s10q.err
