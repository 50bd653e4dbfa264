# distributed parity tests (SimComm ranks on one GPU) + per-rank timing of the P-way split
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1
timeout -k 10 600 python -u tools/dist_timing.py "$@" > gpurun_out/dist_timing.log 2>&1
