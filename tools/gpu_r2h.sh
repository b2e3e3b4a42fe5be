#!/bin/bash
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-r2h}
cd $GRAFT_REPO_ROOT
bash tools/gpu_r2g.sh $TAG || exit 1
bash tools/sq_probe.sh ${TAG}_m1 "RU256 k7d1 fwd" 1 27 || exit 1
bash tools/sq_probe.sh ${TAG}_m0 "RU256 k7d1 fwd" 0 27 || exit 1
