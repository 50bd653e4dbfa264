set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in 1250000 2500000 5000000; do
  timeout -k 10 600 python bench.py --size $s --no-cpu-baseline --no-pmc > gpurun_out/bench_size_$s.json 2> gpurun_out/bench_size_$s.err
done
timeout -k 10 600 python bench.py --dist --no-cpu-baseline --no-pmc --size 1250000 > gpurun_out/bench_dist_1250000.json 2> gpurun_out/bench_dist_1250000.err
