#!/bin/bash
# log-mel change: spectral/glue/c3 tests, frame-kernel times under rocprof, C3 bench x2
set -o pipefail
TAG=${1:-s5d}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_spectral.py tests/test_gpu_glue.py tests/test_gpu_c3.py tests/test_gpu_gan.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
RC=$?; echo "tests rc=$RC"; tail -2 $OUT/${TAG}_tests.log
[ $RC -eq 0 ] || exit 1
CFGS="14=0" bash tools/gpu_s5c.sh ${TAG}p || exit 1
cd $GRAFT_REPO_ROOT
CFGS="0=0 0=0" bash tools/gpu_s3l.sh ${TAG}_c3 || exit 1
