# r03 v17: entries per chunk of the upper-round level loop (CPK_UPPER_CH 8 / 6 builds under abv/,
# default 4): parity with the 8 build, phase cycles (stamps builds), S10 A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
CPK_LIB_PATH=$GRAFT_REPO_ROOT/abv/ch8/libcpk.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r03_v17_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || exit $rc
for v in stamps stamps_ch8 stamps_ch6; do
  CPK_LIB_PATH=$GRAFT_REPO_ROOT/abv/$v/libcpk.so timeout -k 10 300 python -u tools/upper_cycles.py > gpurun_out/r03_v17_upper_cycles_$v.log 2>&1
  rc=$?; echo "$v rc $rc"; [ $rc -eq 0 ] || exit $rc
done
bash tools/gpu_ab2.sh base ch8 ch6 base2 ch8b:CPK_LIB_PATH=$GRAFT_REPO_ROOT/abv/ch8/libcpk.so || exit $?
