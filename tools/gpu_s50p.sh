# GPU tests + rocprof kernel trace of a 10M S50-shaped run
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rm -rf gpurun_out/prof50
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof50 -o s50 -- python3 bench.py --config s50 --size 10000000 --steps 2 --no-cpu-baseline --no-pmc --profile-reps 1 > gpurun_out/prof50.json 2>/dev/null
