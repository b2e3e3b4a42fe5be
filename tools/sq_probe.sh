#!/bin/bash
# SQ counters (3 passes) for tools/ws_probe.py on one shape / mode / variant.
# usage: tools/sq_probe.sh <tag> "<shape name>" <mode> <variant>
set -o pipefail
TAG=$1; SHP=$2; MODE=$3; VAR=$4
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for SET in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d $OUT/${TAG}_p$i -o run -- \
    python $GRAFT_REPO_ROOT/tools/ws_probe.py "$SHP" $MODE $VAR > $OUT/${TAG}_p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $OUT/${TAG}_p$i.log; exit 1; }
done
python $GRAFT_REPO_ROOT/tools/pmc_sq.py $(find $OUT/${TAG}_p1 $OUT/${TAG}_p2 $OUT/${TAG}_p3 -name "*counter_collection.csv") > $OUT/${TAG}_sq.md
find $OUT/${TAG}_p1 $OUT/${TAG}_p2 $OUT/${TAG}_p3 -name "*counter_collection.csv" -delete
grep -E "k_conv" $OUT/${TAG}_sq.md | cut -c1-900
