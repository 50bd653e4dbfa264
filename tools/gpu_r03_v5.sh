# r03 v5: grouped forward levels (lanes per row at narrow levels, DPP-shifted ordered sums):
# parity (parity file, dist refactor), A/B against CPK_LEVEL_GROUP=0
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -q -m "gpu and not slow" -k "parity or refactor or sweep or fused or assignment or apply_bitexact" --timeout 300 --timeout-method thread > gpurun_out/r03_v5_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_ab2.sh base grp0 base2 || exit $?
