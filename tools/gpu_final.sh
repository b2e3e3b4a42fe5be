#!/bin/bash
# Round-end GPU session: full parity suite, smoke, default bench (C3 + fp32
# companion + CPU baseline), C5 bench, C3 kernel stats.  usage: tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-final}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
RC=$?; echo "tests rc=$RC"; tail -2 $OUT/${TAG}_tests.log
[ $RC -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1 || exit 1
tail -1 $OUT/${TAG}_smoke.log
timeout -k 10 500 python bench.py > $OUT/${TAG}_bench.log 2>&1 || exit 1
tail -1 $OUT/${TAG}_bench.log | cut -c1-400
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/${TAG}_c5_bench.log 2>&1 || exit 1
tail -1 $OUT/${TAG}_c5_bench.log | cut -c1-300
bash tools/gpu_r2u.sh ${TAG}_c3 > /dev/null 2>&1 || exit 1
head -4 $OUT/${TAG}_c3_kernel_stats.md
