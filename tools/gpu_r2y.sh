#!/bin/bash
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-r2y}
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_glue.py tests/test_gpu_gan.py tests/test_gpu_model.py tests/test_gpu_conv.py -q -m gpu --timeout 300 --timeout-method thread -rf > $OUT/${TAG}_tests.log 2>&1
RC=$?; echo "tests rc=$RC"; grep -E "passed|failed|FAIL|Error" $OUT/${TAG}_tests.log | tail -12
[ $RC -le 1 ] || exit $RC
timeout -k 10 300 python bench.py --no-fp32-companion --no-cpu-baseline > $OUT/${TAG}_bench.log 2>&1 || { echo "bench failed"; tail -5 $OUT/${TAG}_bench.log; exit 1; }
tail -1 $OUT/${TAG}_bench.log | cut -c1-250
bash tools/gpu_r2u.sh ${TAG} | grep -E "per step|k_pack|k_ru32"
