# r03 v35: distributed construction with parallel index fills, coupling check and Kp slice (no
# Kp copy), sub-phases under CPK_TIMING; single GPU: Kp uploaded in the analysis hook too.
# Parity / factor / boundary / distributed tests, S10 construction phases, one rank's share at P = 8
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/v35
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_factor.py tests/test_gpu_boundary.py tests/test_gpu_dist.py > gpurun_out/v35/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || exit $rc
CPK_TIMING=1 timeout -k 10 300 python -u tools/ptime.py > gpurun_out/v35/ptime.log 2>&1
rc=$?; echo "ptime rc $rc"; [ $rc -eq 0 ] || exit $rc
CPK_TIMING=1 timeout -k 10 300 python -u tools/dist_timing.py 8:0 > gpurun_out/v35/dist_timing.log 2>&1
echo "dist rc $?"
