#!/bin/bash
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 200 --timeout-method thread -rf -s > $OUT/r2d_tests.log 2>&1
RC=$?; echo "tests rc=$RC"; grep -E "passed|failed|FAIL|C3 |RVQ full|bit_cast" $OUT/r2d_tests.log | tail -20
[ $RC -le 1 ] || exit $RC
SHAPE="RU128 k7d9" timeout -k 10 120 python tools/conv_bench.py 0 21 22 23 24 25 26 > $OUT/r2d_cb1.log 2>&1; cat $OUT/r2d_cb1.log
SHAPE="RU256 k7" timeout -k 10 120 python tools/conv_bench.py 0 21 22 23 24 25 26 > $OUT/r2d_cb2.log 2>&1; cat $OUT/r2d_cb2.log
bash tools/sq_conv.sh r2d_sq128 "RU128 k7d9 fwd" 24 || exit 1
bash tools/sq_conv.sh r2d_sq256 "RU256 k7d1 fwd" 24 || exit 1
