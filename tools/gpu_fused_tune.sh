# round-0 staging configurations with the fused refinement residual (S10), fused vs separate
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/tune_sweep.py 192,576,64,1024,4096,512 256,768,64,1024,4096,512 256,768,128,1024,4096,512 384,1152,64,1024,4096,512 > gpurun_out/fused_tune.log 2>&1
CPK_NO_FUSED_RESID=1 timeout -k 10 300 python -u tools/tune_sweep.py 192,576,64,1024,4096,512 256,768,64,1024,4096,512 >> gpurun_out/fused_tune.log 2>&1
