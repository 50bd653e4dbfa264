# per-rank timing of a P-way split for library variants (libcpk_<v>.so)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
RUNS=${RUNS:-8:0}
for v in "$@"; do
  if [ "$v" = default ]; then lib=cpkrylov_amd/libcpk.so; else lib=cpkrylov_amd/libcpk_$v.so; fi
  echo "== $v" >> gpurun_out/dist_ab.log
  CPK_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u tools/dist_timing.py $RUNS 2>&1 | grep "^{" >> gpurun_out/dist_ab.log
done
