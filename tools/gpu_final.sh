#!/bin/bash
# Round-end GPU session: full parity suite, smoke, default bench (C3 + fp32
# companion + CPU baseline), C5 bench (with its CPU baseline), C3 and C5 kernel
# stats.  usage: tools/gpu_final.sh TAG   (each step stops the session on failure)
set -o pipefail
TAG=${1:-final}
cd $GRAFT_REPO_ROOT
bash tools/gpu.sh tests ${TAG} || exit 1
bash tools/gpu.sh smoke ${TAG} || exit 1
bash tools/gpu.sh bench ${TAG} || exit 1
bash tools/gpu.sh bench ${TAG}_c5 --config c5 --steps 10 --warmup 2 || exit 1
bash tools/gpu.sh prof ${TAG}_c3 --steps 5 --warmup 2 > /dev/null || exit 1
STEPS_PROF=4 bash tools/gpu.sh prof ${TAG}_c5 --config c5 --steps 3 --warmup 1 > /dev/null || exit 1
head -8 $GRAFT_REPO_ROOT/gpurun_out/${TAG}_c3_kernel_stats.md
