#!/bin/bash
# C5 kernel stats of the current tree.  usage: tools/gpu_s3s.sh TAG
set -o pipefail
TAG=${1:-s3s}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_c5prof -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/${TAG}_c5prof.log 2>&1 || { echo "c5 prof failed"; exit 1; }
python $GRAFT_REPO_ROOT/tools/prof_summary.py $OUT/${TAG}_c5prof 4 > $OUT/${TAG}_c5_kernel_stats.md
head -32 $OUT/${TAG}_c5_kernel_stats.md | cut -c1-150
