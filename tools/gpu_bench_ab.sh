# bench.py (S10, no CPU baseline / PMC) for library variants (libcpk_<v>.so)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = default ]; then lib=cpkrylov_amd/libcpk.so; else lib=cpkrylov_amd/libcpk_$v.so; fi
  echo "== $v" >> gpurun_out/bench_ab.log
  CPK_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc ${BENCH_ARGS:-} 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['iters_per_step'], d['kernels']['apply']['avg_ms'])" >> gpurun_out/bench_ab.log
done
