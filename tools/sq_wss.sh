#!/bin/bash
# SQ counters of the sample-tile kernel against k_conv_ws_bf16 on the RU256 k7
# shapes (tools/conv_bench.py variants 27 / 50), one rocprofv3 pass per set.
# usage: tools/sq_wss.sh TAG
set -o pipefail
TAG=${1:-wss}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for SET in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU"; do
  i=$((i+1))
  SHAPE="RU256 k7" timeout -k 10 120 rocprofv3 --pmc $SET --output-format csv -d $OUT/${TAG}_p$i -o run -- \
    python $GRAFT_REPO_ROOT/tools/conv_bench.py 27 50 > $OUT/${TAG}_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/${TAG}_p$i.log; exit 1; }
done
python $GRAFT_REPO_ROOT/tools/pmc_sq.py $(find $OUT/${TAG}_p1 $OUT/${TAG}_p2 -name "*counter_collection.csv") > $OUT/${TAG}_sq.md
find $OUT/${TAG}_p1 $OUT/${TAG}_p2 -name "*counter_collection.csv" -delete
cat $OUT/${TAG}_sq.md | grep -v pack_many | cut -c1-600
