#!/bin/bash
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-r2i}
cd $GRAFT_REPO_ROOT
bash tools/gpu_r2g.sh $TAG ${2:-0,1,4} || exit 1
timeout -k 10 120 python tools/ws_probe.py stamps 2>&1 | grep -v amdgpu.ids
