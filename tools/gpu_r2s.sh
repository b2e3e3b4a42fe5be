#!/bin/bash
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-r2s}
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -q -m gpu -k "resunit or residual" --timeout 200 --timeout-method thread -rf > $OUT/${TAG}_tests.log 2>&1
RC=$?; echo "tests rc=$RC"; grep -E "passed|failed|FAIL|Error|assert" $OUT/${TAG}_tests.log | tail -20
exit $RC
