#!/bin/bash
# shortx window prefetch: dconv/GAN tests, then C5 A/B against tune 34 = 1
set -o pipefail
TAG=${1:-s5g}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_dconv_variants.py tests/test_gpu_gan.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
RC=$?; echo "tests rc=$RC"; tail -2 $OUT/${TAG}_tests.log
[ $RC -eq 0 ] || exit 1
ENVS="SEL_TUNE=34=1 SEL_TUNE=34=0 SEL_TUNE=34=1 SEL_TUNE=34=0" bash tools/gpu_s4d.sh ${TAG}
