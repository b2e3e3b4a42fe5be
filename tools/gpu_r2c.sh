#!/bin/bash
# GAN / glue / spectral-probe tests, then the spilling-build A/B of the spectral
# tests (SEL_LIB=libsel_w4.so), then the C5 bench.
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_gan.py tests/test_gpu_glue.py tests/test_gpu_spectral.py -q -m gpu \
  --timeout 200 --timeout-method thread -rf -s > $OUT/r2c_tests.log 2>&1
RC=$?; echo "tests rc=$RC"; grep -E "passed|failed|b64|FAIL" $OUT/r2c_tests.log | tail -15
[ $RC -le 1 ] || exit $RC
SEL_LIB=$GRAFT_REPO_ROOT/dl-speech-enhancement_amd/sel/libsel_w4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_spectral.py -q -m gpu \
  --timeout 120 --timeout-method thread -rf > $OUT/r2c_w4.log 2>&1
RC=$?; echo "w4 rc=$RC"; grep -E "passed|failed|FAIL" $OUT/r2c_w4.log | tail -12
[ $RC -le 1 ] || exit $RC
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 > $OUT/r2c_c5.log 2>&1
echo "c5 rc=$?"; tail -2 $OUT/r2c_c5.log
