# r03 v9: grouped levels in the upper-round / last-round kernels; construction without zero
# uploads, parallel intra-block levels: parity, A/B against CPK_UPPER_GROUP=0, construction time
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_factor.py -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/r03_v9_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_ab2.sh base ugrp0 base2 || exit $?
timeout -k 10 600 python -u tools/ptime.py > gpurun_out/r03_v9_ptime.log 2>&1
echo "ptime rc $?"
