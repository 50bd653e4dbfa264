# fused refinement residual: parity, round-0 staging configurations (S10), tail rows in-kernel vs a launch
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "fused" --timeout 120 --timeout-method thread > gpurun_out/fused2_parity.log 2>&1
timeout -k 10 400 python -u tools/tune_sweep.py 192,576,64,1024,4096,512 256,768,64,1024,4096,512 256,768,128,1024,4096,512 384,1152,64,1024,4096,512 > gpurun_out/fused_tune.log 2>&1
CPK_FUSED_TAIL_LAUNCH=1 timeout -k 10 300 python -u tools/tune_sweep.py 192,576,64,1024,4096,512 >> gpurun_out/fused_tune.log 2>&1
CPK_NO_FUSED_RESID=1 timeout -k 10 300 python -u tools/tune_sweep.py 192,576,64,1024,4096,512 >> gpurun_out/fused_tune.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/fused2_b.json 2> gpurun_out/fused2_b.err
