# round-3 validation: the default S10 bench line (PMC passes + CPU baseline), the rocprofv3 kernel
# trace of the same bench command, the S50 bench line, smoke
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 420 python bench.py > gpurun_out/final/bench_s10.json 2> gpurun_out/final/bench_s10.err
rc=$?; echo "bench rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof -o bench -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/final/prof_bench.json 2> gpurun_out/final/prof_bench.err
rc=$?; echo "rocprof rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py --config s50 --no-cpu-baseline > gpurun_out/final/bench_s50.json 2> gpurun_out/final/bench_s50.err
rc=$?; echo "s50 rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1
echo "smoke rc $?"
