# r03 v38 (diagnostic): the first forward sweep's input through perm vs already in schedule order
# (engine option profile_fwd_sched: cpk_profile_kernels' forward reads x as the schedule-order
# input, no perm gather). S10 bench with its PMC passes, each way, no CPU baseline.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/v38
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/v38/perm.json 2> gpurun_out/v38/perm.err
rc=$?; echo "bench perm rc $rc"; [ $rc -eq 0 ] || exit $rc
CPK_PROFILE_FWD_SCHED=1 timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/v38/sched.json 2> gpurun_out/v38/sched.err
echo "bench sched rc $?"
