set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rm -rf gpurun_out/prof_small
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_small -o small -- python3 bench.py --size 1250000 --steps 3 --no-cpu-baseline --no-pmc --profile-reps 2 > gpurun_out/prof_small.json 2> gpurun_out/prof_small.err
timeout -k 10 600 python bench.py --no-cpu-baseline --no-pmc > gpurun_out/bench_s10q.json 2> gpurun_out/bench_s10q.err
