set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 600 python bench.py --size 1000000 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_1m.json 2> gpurun_out/bench_1m.err
timeout -k 10 900 python bench.py > gpurun_out/bench_s10.json 2> gpurun_out/bench_s10.err
