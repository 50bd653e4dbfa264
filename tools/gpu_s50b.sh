# S50 at 50M: the bench line (120 iterations per step) and one run to convergence
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --config s50 --steps 3 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/s50_bench.json 2> gpurun_out/s50_bench.err
timeout -k 10 600 python bench.py --config s50 --itmax 3000 --steps 1 --warmup 0 --no-cpu-baseline --no-pmc > gpurun_out/s50_conv.json 2> gpurun_out/s50_conv.err
