# bisect the distributed apply tests over tree snapshots under tools/ab
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in tools/ab/t_*; do
  (cd $t && timeout -k 10 120 python -u -m pytest tests/test_gpu_dist.py -q -k "test_dist_apply_bitexact and cvxqp1_m" --timeout 60 --timeout-method thread > $GRAFT_REPO_ROOT/gpurun_out/dist_$(basename $t).log 2>&1)
  echo "$t rc=$?"
done
