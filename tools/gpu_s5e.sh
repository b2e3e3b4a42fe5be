#!/bin/bash
# two-chunks-per-barrier ws (K = 2): conv/dconv/GAN tests (default, and the
# generator's K = 2 layers on ws via tune 27), then C5 A/B against tune 33 = 1
set -o pipefail
TAG=${1:-s5e}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_dconv_variants.py tests/test_gpu_gan.py tests/test_gpu_conv.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
RC=$?; echo "tests rc=$RC"; tail -2 $OUT/${TAG}_tests.log
[ $RC -eq 0 ] || exit 1
SEL_TUNE=27=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_c3.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/${TAG}_tests27.log 2>&1
RC=$?; echo "tests27 rc=$RC"; tail -2 $OUT/${TAG}_tests27.log
[ $RC -eq 0 ] || exit 1
ENVS="SEL_TUNE=33=1 SEL_TUNE=33=0 SEL_TUNE=33=1 SEL_TUNE=33=0" bash tools/gpu_s4d.sh ${TAG}
