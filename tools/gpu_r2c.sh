# round 2: sweep configuration sweep at S10 (round 0 varied, upper rounds at the default), rocprof of the bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
U=1024,4096,512
CPK_NO_DETACH=1 timeout -k 10 300 python -u tools/tune_sweep.py 192,576,64,$U > gpurun_out/tune.log 2>&1
timeout -k 10 600 python -u tools/tune_sweep.py 192,576,64,$U 256,768,64,$U 256,768,128,$U 128,384,64,$U 128,512,128,$U 384,1152,64,$U >> gpurun_out/tune.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 5 --no-cpu-baseline --no-pmc > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
