# A/B of library variants and engine options: each argument is name[:ENV=VALUE[+ENV=VALUE]];
# a name with a build under abx/<name>/ uses that libcpk.so, otherwise the in-tree one.
# S10 bench (it/s) and the rocprofv3 kernel stats of the same command, per variant
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for spec in "$@"; do
  v=${spec%%:*}
  envs=""
  [ "$spec" != "$v" ] && envs=${spec#*:}
  lib=$GRAFT_REPO_ROOT/cpkrylov_amd/libcpk.so
  [ -f abx/$v/libcpk.so ] && lib=$GRAFT_REPO_ROOT/abx/$v/libcpk.so
  ( export CPK_LIB_PATH=$lib; for kv in ${envs//+/ }; do export "$kv"; done
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/$v -o p -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err ) || exit $?
  echo "$v done"
done
