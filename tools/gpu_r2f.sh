#!/bin/bash
# warp-specialised conv kernel: parity (tile-variant test) + microbench A/B
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-r2f}
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_c3.py -q -m gpu -k "tile_variants" --timeout 200 --timeout-method thread -rf > $OUT/${TAG}_tests.log 2>&1
RC=$?; echo "tests rc=$RC"; grep -E "passed|failed|FAIL|Error" $OUT/${TAG}_tests.log | tail -8
[ $RC -le 1 ] || exit $RC
SHAPE=RU256 timeout -k 10 200 python tools/conv_bench.py 0 24 27 > $OUT/${TAG}_cb1.log 2>&1 || exit 1
SHAPE=down2 timeout -k 10 200 python tools/conv_bench.py 0 24 27 >> $OUT/${TAG}_cb1.log 2>&1 || exit 1
cat $OUT/${TAG}_cb1.log | grep -v amdgpu.ids
