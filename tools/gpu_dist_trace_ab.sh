# kernel traces of one rank's share of a P-way solve (CPK_COMM=null) for library variants
# (libcpk_<v>.so; "default" = libcpk.so); summaries in gpurun_out/dtrace_<v>.txt
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
RUNS=${RUNS:-8:0}
for v in "$@"; do
  if [ "$v" = default ]; then lib=cpkrylov_amd/libcpk.so; else lib=cpkrylov_amd/libcpk_$v.so; fi
  rm -rf gpurun_out/dtrace_$v
  CPK_LIB_PATH=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/dtrace_$v -o dt -- python3 tools/dist_timing.py $RUNS > gpurun_out/dtrace_$v.log 2>&1
  python3 tools/prof_summary.py gpurun_out/dtrace_$v/dt_kernel_trace.csv 3 > gpurun_out/dtrace_$v.txt
done
