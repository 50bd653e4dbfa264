# A/B of libcpk.so variants (abx/<name>/) on S50 at 10M dofs: kernel trace per variant
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab50
export TMPDIR=/tmp
for v in base "$@"; do
  lib=$GRAFT_REPO_ROOT/cpkrylov_amd/libcpk.so
  [ -f abx/$v/libcpk.so ] && lib=$GRAFT_REPO_ROOT/abx/$v/libcpk.so
  CPK_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab50/$v -o p -- python3 bench.py --config s50 --size 10000000 --steps 2 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/ab50/$v.json 2> gpurun_out/ab50/$v.err || exit $?
  echo "$v done"
done
