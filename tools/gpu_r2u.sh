#!/bin/bash
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-r2u}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fp32-companion > $OUT/${TAG}_prof.log 2>&1 || { echo "prof failed"; exit 1; }
python $GRAFT_REPO_ROOT/tools/prof_summary.py $OUT/${TAG}_prof 7 > $OUT/${TAG}_kernel_stats.md
head -30 $OUT/${TAG}_kernel_stats.md | cut -c1-200
