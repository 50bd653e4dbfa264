# r03 v24: cpminres update fused into the Lanczos step and the Krylov product (no MinresUpdate
# pass): the bit-exact tests (fused against no_minres_fuse, 1 GPU and SimComm ranks, and the
# cpminres oracle parity cases), then the S10 bench with and without it under rocprofv3
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "minres or reg_cpkrylov" tests/test_gpu_dist.py::test_dist_minres_fused_update_bitexact tests/test_gpu_dist.py::test_dist_minres_merged_exchanges > gpurun_out/r03_v24_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab2.sh fused unfused:CPK_NO_MINRES_FUSE=1 fused2
