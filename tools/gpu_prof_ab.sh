# rocprofv3 kernel trace of a short bench run for library variants (libcpk_<v>.so)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = default ]; then lib=cpkrylov_amd/libcpk.so; else lib=cpkrylov_amd/libcpk_$v.so; fi
  rm -rf gpurun_out/pab_$v
  CPK_LIB_PATH=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pab_$v -o t -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pmc --profile-reps 1 > gpurun_out/pab_$v.json 2>/dev/null
done
