# r03 v18: the distributed bench path under torchrun with one rank (RCCL communicator, captured
# collectives), and one rank's share of the P = 8 split (CPK_COMM=null) on the final code
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dist
export TMPDIR=/tmp
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 1 --dist --steps 5 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/r03_v18_torchrun.json 2> gpurun_out/r03_v18_torchrun.err
rc=$?; echo "torchrun rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/dist_timing.py 1:0 8:0 8:7 > gpurun_out/dist/timing_v18.log 2>&1
echo "dist rc $?"
