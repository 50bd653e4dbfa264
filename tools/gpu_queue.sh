# round-0 block queue (CPK_PIPE_QUEUE) A/B: parity subset both ways, sweep timings, S10 bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "bitexact or fused" --timeout 120 --timeout-method thread > gpurun_out/q_parity_default.log 2>&1
CPK_PIPE_QUEUE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "bitexact or fused" --timeout 120 --timeout-method thread > gpurun_out/q_parity_queue.log 2>&1
timeout -k 10 200 python -u tools/tune_sweep.py 192,576,64,1024,4096,512 > gpurun_out/q_tune.log 2>&1
CPK_PIPE_QUEUE=1 timeout -k 10 200 python -u tools/tune_sweep.py 192,576,64,1024,4096,512 >> gpurun_out/q_tune.log 2>&1
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/q_b0.json 2> gpurun_out/q_b0.err
CPK_PIPE_QUEUE=1 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/q_b1.json 2> gpurun_out/q_b1.err
