#!/bin/bash
# full GPU suite, then C3 (x2) and C5 benches.  usage: tools/gpu_s5b.sh TAG
set -o pipefail
TAG=${1:-s5b}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
RC=$?; echo "tests rc=$RC"; tail -2 $OUT/${TAG}_tests.log
[ $RC -eq 0 ] || exit 1
CFGS="0=0 0=0" bash tools/gpu_s3l.sh ${TAG}_c3 || exit 1
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/${TAG}_c5_bench.log 2>&1 || exit 1
tail -1 $OUT/${TAG}_c5_bench.log | cut -c1-300
