# A/B of libcpk.so variants built under abx/<name>/ (plus the in-tree build as "base"):
# S10 bench (it/s) and the rocprofv3 kernel stats of the same command, per variant
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for v in base "$@" base2; do
  lib=$GRAFT_REPO_ROOT/cpkrylov_amd/libcpk.so
  [ -f abx/$v/libcpk.so ] && lib=$GRAFT_REPO_ROOT/abx/$v/libcpk.so
  CPK_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/$v -o p -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || exit $?
  echo "$v done"
done
