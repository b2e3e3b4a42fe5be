#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/ws_probe.py stamps ${1:-0,1} 2>&1 | grep -v amdgpu.ids
bash tools/gpu_r2m.sh r2n 0
