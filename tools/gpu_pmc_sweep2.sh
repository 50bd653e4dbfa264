# SQ counters of the round-0 sweep kernels at S10 (two passes, filtered to sptrsv_pipe)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  N=${N:-10000000} REPS=3 timeout -k 10 240 rocprofv3 --pmc $P --kernel-include-regex "${KRE:-sptrsv}" --output-format csv -d gpurun_out/pmc2 -o pass$i -- python3 tools/tune_sweep.py ${CFG:-192,576,64,1024,4096,512} > gpurun_out/pmc2/pass$i.log 2>&1
done
