# fused refinement residual: parity file, then an A/B bench (fused vs CPK_NO_FUSED_RESID) on S10
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fused_parity.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/fused_b.json 2> gpurun_out/fused_b.err
CPK_NO_FUSED_RESID=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/fused_b0.json 2> gpurun_out/fused_b0.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fused -o bench -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/fused_prof.json 2> gpurun_out/fused_prof.err
