#!/bin/bash
# SQ counters (2 passes) for an arbitrary python tool.  Usage: tools/sq_cmd.sh <tag> <script.py> [args]
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for SET in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $SET --output-format csv -d $OUT/${TAG}_p$i -o run -- \
    python $GRAFT_REPO_ROOT/"$@" > $OUT/${TAG}_p$i.log 2>&1 || exit 1
done
python $GRAFT_REPO_ROOT/tools/pmc_sq.py $(find $OUT/${TAG}_p1 $OUT/${TAG}_p2 -name "*counter_collection.csv") > $OUT/${TAG}_sq.md
find $OUT/${TAG}_p1 $OUT/${TAG}_p2 -name "*counter_collection.csv" -delete
