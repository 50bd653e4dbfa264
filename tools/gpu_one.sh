set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_dist.py -x -q -m gpu -k "more_ranks" > gpurun_out/pytest_one.log 2>&1
