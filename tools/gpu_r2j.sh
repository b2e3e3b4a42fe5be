#!/bin/bash
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/ws_probe.py stamps ${1:-0,1,16,32,64,96,48} 2>&1 | grep -v amdgpu.ids | grep -v "after one"
timeout -k 10 200 python tools/ws_probe.py "down2 640->256 k3" 0,4 27,24 2>&1 | grep -v amdgpu.ids
