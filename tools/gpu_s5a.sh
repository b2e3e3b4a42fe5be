#!/bin/bash
# ws consumer-layout A/B: conv parity tests under SEL_TUNE=32=1, then C3 alternating.
set -o pipefail
TAG=${1:-s5a}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
SEL_TUNE=32=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_dconv_variants.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
RC=$?; echo "tests rc=$RC"; tail -2 $OUT/${TAG}_tests.log
[ $RC -eq 0 ] || exit 1
CFGS="${CFGS:-0=0 32=1 0=0 32=1}" bash tools/gpu_s3l.sh ${TAG}
