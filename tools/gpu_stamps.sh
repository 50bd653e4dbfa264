# round-0 sweep tail measurement with the stamp-instrumented library (abx/stamps)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
CPK_LIB_PATH=$GRAFT_REPO_ROOT/abx/stamps/libcpk.so timeout -k 10 300 python -u tools/pipe_stamps.py > gpurun_out/stamps.log 2>&1
