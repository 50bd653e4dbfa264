# round-3 validation of the final code: the driver's GPU suite command (timed), then the
# default S10 bench line with PMC + CPU baseline, its rocprofv3 kernel trace, smoke
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final2
export TMPDIR=/tmp
s=$(date +%s)
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 600 --timeout-method thread --durations=15 > gpurun_out/final2/pytest.log 2>&1
rc=$?; echo "pytest rc $rc wall $(( $(date +%s) - s )) s"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py > gpurun_out/final2/bench_s10.json 2> gpurun_out/final2/bench_s10.err
rc=$?; echo "bench rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final2/prof -o bench -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/final2/prof_bench.json 2> gpurun_out/final2/prof_bench.err
rc=$?; echo "rocprof rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final2/smoke.log 2>&1
echo "smoke rc $?"
