# S50: window-pass variants (CPK_DOT_GROUP) with a kernel trace each, at 10M dofs
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q -k "dqgmres or gmres" --timeout 120 --timeout-method thread > gpurun_out/s50_parity.log 2>&1
for g in 16 24 48; do
  CPK_DOT_GROUP=$g timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof50_$g -o s50 -- python3 bench.py --config s50 --size 10000000 --steps 2 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/s50_g$g.json 2> gpurun_out/s50_g$g.err
done
