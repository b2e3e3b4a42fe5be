#!/bin/bash
# conv kernel iteration: parity (tile-variant test) + diagnostic probe
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-r2g}
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_c3.py -q -m gpu -k "tile_variants" --timeout 200 --timeout-method thread -rf > $OUT/${TAG}_tests.log 2>&1
RC=$?; echo "tests rc=$RC"; grep -E "passed|failed|FAIL|Error" $OUT/${TAG}_tests.log | tail -8
[ $RC -le 1 ] || exit $RC
timeout -k 10 200 python tools/ws_probe.py "RU256 k7d1 fwd,RU256 k7 dgrad,down2 640->256 k3" ${2:-0,1,2,4} 27,24 2>&1 | grep -v amdgpu.ids
