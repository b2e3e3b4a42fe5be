#!/bin/bash
# SQ counter passes (one rocprofv3 run each) on the STFT |X| kernel alone (tools/stft_one.py)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/sqs
cd /tmp && export TMPDIR=/tmp
i=0
for C in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/sqs/p$i -o run -- python $GRAFT_REPO_ROOT/tools/stft_one.py ${STFT_ARGS:-} > $GRAFT_REPO_ROOT/gpurun_out/sqs/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $GRAFT_REPO_ROOT/gpurun_out/sqs/p$i.log; exit 1; }
done
cd $GRAFT_REPO_ROOT
python tools/pmc_sq.py $(find gpurun_out/sqs -name "*counter_collection.csv") | tee gpurun_out/sqs/summary.md
