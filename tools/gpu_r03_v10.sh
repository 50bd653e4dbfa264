# r03 v10: XCD-affine round-0 assignment (engine option r0_xcd_chunk): parity, A/B against the
# plain assignment, and the PMC traffic of both
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 240 --timeout-method thread -k "assignment or fused_last" > gpurun_out/r03_v10_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab2.sh base xcd16:CPK_R0_XCD_CHUNK=16 xcd4:CPK_R0_XCD_CHUNK=4 xcd64:CPK_R0_XCD_CHUNK=64 base2 || exit $?
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r03_v10_pmc_base.json 2> gpurun_out/r03_v10_pmc_base.err || exit $?
echo "pmc base done"
CPK_R0_XCD_CHUNK=16 timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r03_v10_pmc_xcd16.json 2> gpurun_out/r03_v10_pmc_xcd16.err || exit $?
echo "pmc xcd16 done"
