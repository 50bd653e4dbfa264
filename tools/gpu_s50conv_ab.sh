# S50 at 50M run to convergence with a variant library (abx/<name>/libcpk.so) and the in-tree one
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in "$@"; do
  CPK_LIB_PATH=$GRAFT_REPO_ROOT/abx/$v/libcpk.so timeout -k 10 600 python bench.py --config s50 --itmax 3000 --steps 1 --warmup 0 --no-cpu-baseline --no-pmc > gpurun_out/s50_conv_$v.json 2> gpurun_out/s50_conv_$v.err
done
