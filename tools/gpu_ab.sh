# A/B of library variants under tools/ab (CPK_LIB_PATH) on the S10 sweep profile
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
U=192,576,64,1024,4096,512
timeout -k 10 200 python -u tools/tune_sweep.py $U > gpurun_out/ab.log 2>&1
for l in tools/ab/*.so; do
  echo "== $l" >> gpurun_out/ab.log
  CPK_LIB_PATH=$GRAFT_REPO_ROOT/$l timeout -k 10 200 python -u tools/tune_sweep.py $U >> gpurun_out/ab.log 2>&1
done
