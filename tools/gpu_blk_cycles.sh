# per-block cycles of the round-0 sweep variants (library built with -DCPK_PIPE_STAMPS under
# abx/stamps/): the round-0 cost model of the LPT block assignment
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
CPK_LIB_PATH=$GRAFT_REPO_ROOT/abx/stamps/libcpk.so timeout -k 10 300 python -u tools/blk_cycles.py > gpurun_out/blk_cycles.log 2>&1
CPK_LIB_PATH=$GRAFT_REPO_ROOT/abx/stamps/libcpk.so timeout -k 10 300 python -u tools/pipe_stamps.py > gpurun_out/stamps.log 2>&1
