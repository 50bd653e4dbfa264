# r03 v37: distributed construction without the global schedule / relabelling (each rank
# schedules its own subtrees) and split_tree's parallel passes: distributed tests, then one
# rank's share at P = 8 (construction phases under CPK_TIMING)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/v37
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_boundary.py > gpurun_out/v37/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || exit $rc
CPK_TIMING=1 timeout -k 10 300 python -u tools/dist_timing.py 8:0 > gpurun_out/v37/dist_timing.log 2>&1
echo "dist rc $?"
