# r03 v14: phase cycles of the upper-round blocks (stamps build, tools/upper_cycles.py), and an
# S10 A/B of smaller upper-round blocks (second staging triple of the sweep option)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
CPK_LIB_PATH=$GRAFT_REPO_ROOT/abv/stamps/libcpk.so timeout -k 10 300 python -u tools/upper_cycles.py > gpurun_out/r03_v14_upper_cycles.log 2>&1
rc=$?; echo "upper_cycles rc $rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab2.sh base up512:CPK_SWEEP=192,576,64,512,2048,512 up256:CPK_SWEEP=192,576,64,256,1024,512 base2 || exit $?
