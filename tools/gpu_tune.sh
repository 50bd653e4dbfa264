# sweep timings at S10 for the staging configurations given as arguments (tune_sweep.py)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/tune_sweep.py "$@" > gpurun_out/tune.log 2>&1
