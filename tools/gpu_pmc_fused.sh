# S10 bench with its PMC passes (the fused residual sweep's traffic included), no CPU baseline
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_pmc.json 2> gpurun_out/bench_pmc.err
