set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_dist.py -x -q -m gpu > gpurun_out/pytest_dist.log 2>&1
timeout -k 10 600 python bench.py --dist --no-cpu-baseline --no-pmc > gpurun_out/bench_dist1.json 2> gpurun_out/bench_dist1.err
timeout -k 10 600 python bench.py --no-cpu-baseline --no-pmc > gpurun_out/bench_single.json 2> gpurun_out/bench_single.err
