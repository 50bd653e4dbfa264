# r02 v5: S50 bench line (the fused refinement residual applies to its preconditioner too) and the
# headline-size parity file (S10 / S50, one GPU and 8 simulated ranks)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config s50 --steps 3 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/s50_bench.json 2> gpurun_out/s50_bench.err
timeout -k 10 800 python -u -m pytest tests/test_gpu_scale.py -x -v --timeout 780 --timeout-method thread > gpurun_out/scale_all.log 2>&1
