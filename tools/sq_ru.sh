#!/bin/bash
# SQ counters of the fused residual-unit kernels (tools/ru_bench.py at C3 size,
# 32- and 64-channel units), one rocprofv3 pass per counter set.
# usage: tools/sq_ru.sh TAG
set -o pipefail
TAG=${1:-ru}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for SET in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU"; do
  i=$((i+1))
  for C in 32 64; do
    RU_C=$C timeout -k 10 200 rocprofv3 --pmc $SET --output-format csv -d $OUT/${TAG}_c${C}_p$i -o run -- \
      python $GRAFT_REPO_ROOT/tools/ru_bench.py > $OUT/${TAG}_c${C}_p$i.log 2>&1 || { echo "pass $i C$C failed"; tail -5 $OUT/${TAG}_c${C}_p$i.log; exit 1; }
  done
done
python $GRAFT_REPO_ROOT/tools/pmc_sq.py $(find $OUT/${TAG}_c*_p1 $OUT/${TAG}_c*_p2 -name "*counter_collection.csv") > $OUT/${TAG}_sq.md
find $OUT/${TAG}_c*_p1 $OUT/${TAG}_c*_p2 -name "*counter_collection.csv" -delete
grep -E "k_ru" $OUT/${TAG}_sq.md | cut -c1-700
