# distributed path at one rank (1-rank RCCL) vs the single-GPU path, S10
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc > gpurun_out/b_single.json 2> gpurun_out/b_single.err
timeout -k 10 300 python bench.py --dist --no-cpu-baseline --no-pmc > gpurun_out/b_dist1.json 2> gpurun_out/b_dist1.err
