set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 900 python bench.py --config s50 --steps 3 > gpurun_out/bench_s50.json 2> gpurun_out/bench_s50.err
