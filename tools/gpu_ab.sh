# A/B of library variants (libcpk_<v>.so next to libcpk.so): sweep/apply timings at S10, parity of the default build
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1
CFG=${CFG:-192,576,64,1024,4096,512}
for v in ${@:-v0 default}; do
  if [ "$v" = default ]; then lib=cpkrylov_amd/libcpk.so; else lib=cpkrylov_amd/libcpk_$v.so; fi
  echo "== $v" >> gpurun_out/ab.log
  CPK_LIB_PATH=$PWD/$lib N=${N:-10000000} timeout -k 10 300 python -u tools/tune_sweep.py $CFG >> gpurun_out/ab.log 2>&1
done
