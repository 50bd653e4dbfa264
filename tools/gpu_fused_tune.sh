# fused refinement residual: round-0 staging configurations (S10), in-kernel tail rows vs a launch,
# separate residual; then the S10 headline-size parity test
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/tune_sweep.py 192,576,64,1024,4096,512 256,768,64,1024,4096,512 256,768,128,1024,4096,512 384,1152,64,1024,4096,512 > gpurun_out/fused_tune.log 2>&1
CPK_FUSED_TAIL_LAUNCH=1 timeout -k 10 200 python -u tools/tune_sweep.py 192,576,64,1024,4096,512 >> gpurun_out/fused_tune.log 2>&1
CPK_NO_FUSED_RESID=1 timeout -k 10 200 python -u tools/tune_sweep.py 192,576,64,1024,4096,512 256,768,64,1024,4096,512 >> gpurun_out/fused_tune.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -x -v -k "s10_one_gpu" --timeout 580 --timeout-method thread > gpurun_out/scale_s10.log 2>&1
