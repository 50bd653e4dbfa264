# Interleaved A/B of library builds (abx/<name>/libcpk.so; "base" = the in-tree build) and
# engine options as environment variables: name[:ENV=VALUE[+ENV=VALUE]].  Each round runs every
# variant once (bench.py, no profiler), ROUNDS rounds (default 2), so box drift hits every arm
# alike; BENCH_ARGS overrides the bench arguments (default: the +-64 headline, no side blocks).
# Output: gpurun_out/abw/<variant>.<round>.json
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abw
export TMPDIR=/tmp
ROUNDS=${ROUNDS:-2}
ARGS=${BENCH_ARGS:---steps 10 --warmup 2 --no-cpu-baseline --no-pmc --no-exact --no-sub}
for r in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    v=${spec%%:*}
    envs=""
    [ "$spec" != "$v" ] && envs=${spec#*:}
    lib=$GRAFT_REPO_ROOT/cpkrylov_amd/libcpk.so
    [ -f abx/$v/libcpk.so ] && lib=$GRAFT_REPO_ROOT/abx/$v/libcpk.so
    ( export CPK_LIB_PATH=$lib; for kv in ${envs//+/ }; do export "$kv"; done
      timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/abw/$v.$r.json 2> gpurun_out/abw/$v.$r.err ) || exit $?
    echo "[$(date +%T)] $v round $r: $(python3 -c "import json,sys; d=json.load(open('gpurun_out/abw/$v.$r.json')); print(d['value'], d['roofline']['frac'])")"
  done
done
