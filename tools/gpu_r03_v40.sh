# r03 v40: round-0 subtree cap 480 with 256-thread upper-round blocks of <= 512 rows / 3072 entries
# (a 38 KB image: the 1024 round-1 blocks co-resident). Parity file under that configuration, then
# the S10 bench A/B under rocprofv3.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/v40
export TMPDIR=/tmp
CPK_SWEEP=192,576,64,512,3072,256,480 timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/v40/pytest_n256.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab2.sh base n256:CPK_SWEEP=192,576,64,512,3072,256,480 base2 n256b:CPK_SWEEP=192,576,64,512,3072,256,480
