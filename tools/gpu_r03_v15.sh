# r03 v15: grouped levels in the forward upper rounds only (CPK_UPPER_GROUP_FWD=1 builds under
# abv/): phase cycles of the upper blocks with and without (stamps builds), the S10 A/B of the
# same switch, and smaller upper-round blocks (second staging triple of the sweep option)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
CPK_LIB_PATH=$GRAFT_REPO_ROOT/abv/stamps/libcpk.so timeout -k 10 300 python -u tools/upper_cycles.py > gpurun_out/r03_v15_upper_cycles.log 2>&1
rc=$?; echo "upper_cycles rc $rc"; [ $rc -eq 0 ] || exit $rc
CPK_LIB_PATH=$GRAFT_REPO_ROOT/abv/stamps_ugf/libcpk.so timeout -k 10 300 python -u tools/upper_cycles.py > gpurun_out/r03_v15_upper_cycles_ugf.log 2>&1
rc=$?; echo "upper_cycles ugf rc $rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab2.sh base ugf base2 ugf2:CPK_LIB_PATH=$GRAFT_REPO_ROOT/abv/ugf/libcpk.so up512:CPK_SWEEP=192,576,64,512,2048,512 up256:CPK_SWEEP=192,576,64,256,1024,512 || exit $?
