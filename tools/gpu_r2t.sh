#!/bin/bash
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-r2t}
cd $GRAFT_REPO_ROOT
bash tools/gpu_r2s.sh ${TAG}s || exit 1
timeout -k 10 300 python bench.py --no-fp32-companion --no-cpu-baseline > $OUT/${TAG}_bench.log 2>&1 || { echo "bench failed"; tail -5 $OUT/${TAG}_bench.log; exit 1; }
tail -1 $OUT/${TAG}_bench.log | cut -c1-300
SEL_RU_FUSED=0 timeout -k 10 300 python bench.py --no-fp32-companion --no-cpu-baseline > $OUT/${TAG}_bench0.log 2>&1 || { echo "bench0 failed"; exit 1; }
tail -1 $OUT/${TAG}_bench0.log | cut -c1-300
timeout -k 10 300 python bench.py --no-fp32-companion --no-cpu-baseline > $OUT/${TAG}_bench2.log 2>&1 || { echo "bench failed"; exit 1; }
tail -1 $OUT/${TAG}_bench2.log | cut -c1-300
