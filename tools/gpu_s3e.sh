#!/bin/bash
# C3 kernel stats + PMC traffic of the current tree.  usage: tools/gpu_s3e.sh TAG
set -o pipefail
TAG=${1:-s3e}
OUT=$GRAFT_REPO_ROOT/gpurun_out
bash $GRAFT_REPO_ROOT/tools/gpu_r2u.sh ${TAG}_c3 > /dev/null 2>&1 || { echo "c3 prof failed"; exit 1; }
head -3 $OUT/${TAG}_c3_kernel_stats.md
bash $GRAFT_REPO_ROOT/tools/pmc_round.sh ${TAG}_pmc || { echo "pmc failed"; exit 1; }
