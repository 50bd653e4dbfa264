# r03 v16: the upper-round level loop reading the next chunk's columns and values during this
# chunk's gathers (CPK_UPPER_PF=1 builds under abv/): parity with that build, phase cycles of
# the upper blocks (stamps build), S10 A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
CPK_LIB_PATH=$GRAFT_REPO_ROOT/abv/upf/libcpk.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r03_v16_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || exit $rc
CPK_LIB_PATH=$GRAFT_REPO_ROOT/abv/stamps_upf/libcpk.so timeout -k 10 300 python -u tools/upper_cycles.py > gpurun_out/r03_v16_upper_cycles_upf.log 2>&1
rc=$?; echo "upper_cycles rc $rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab2.sh base upf base2 upf2:CPK_LIB_PATH=$GRAFT_REPO_ROOT/abv/upf/libcpk.so || exit $?
