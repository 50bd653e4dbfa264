set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_s50
timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_s50 -o s50 -- python3 bench.py --config s50 --size 10000000 --steps 2 --no-cpu-baseline --no-pmc --profile-reps 2 > gpurun_out/prof_s50.json 2> gpurun_out/prof_s50.err
python3 tools/prof_summary.py gpurun_out/prof_s50/s50_kernel_trace.csv > gpurun_out/prof_s50_summary.txt
