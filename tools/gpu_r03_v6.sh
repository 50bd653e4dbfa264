# r03 v6: the last sweep round forward + backward fused: parity, the default bench (PMC
# passes), A/B against no_fuse_last
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_factor.py -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/r03_v6_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python bench.py --no-cpu-baseline > gpurun_out/r03_v6_bench.json 2> gpurun_out/r03_v6_bench.err
rc=$?; echo "bench rc $rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab2.sh base nofuse:CPK_NO_FUSE_LAST=1 base2 || exit $?
