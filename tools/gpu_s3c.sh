#!/bin/bash
# C3 + C5 kernel stats of the current tree (rocprofv3 kernel trace).  usage: tools/gpu_s3c.sh TAG
set -o pipefail
TAG=${1:-s3c}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
bash $GRAFT_REPO_ROOT/tools/gpu_r2u.sh ${TAG}_c3 > /dev/null 2>&1 || { echo "c3 prof failed"; exit 1; }
head -3 $OUT/${TAG}_c3_kernel_stats.md
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_c5prof -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/${TAG}_c5prof.log 2>&1 || { echo "c5 prof failed"; exit 1; }
python $GRAFT_REPO_ROOT/tools/prof_summary.py $OUT/${TAG}_c5prof 4 > $OUT/${TAG}_c5_kernel_stats.md
head -20 $OUT/${TAG}_c5_kernel_stats.md | cut -c1-160
