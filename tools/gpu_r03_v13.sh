# r03 v13: the cooperative upper-round launch (engine option upper_chain): parity and S10 A/B;
# then the round-3 validation (tools/gpu_r03_final.sh)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 240 --timeout-method thread -k "fused_last or assignment" > gpurun_out/r03_v13_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab2.sh base chain:CPK_UPPER_CHAIN=1 || exit $?
bash tools/gpu_r03_final.sh
