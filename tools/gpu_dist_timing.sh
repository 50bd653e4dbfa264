set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/dist_timing.py "$@" > gpurun_out/dist_timing.log 2>&1
