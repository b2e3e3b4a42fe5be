#!/bin/bash
# C3 with the warp-specialised conv as default: parity + bench + kernel stats
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-r2r}
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_conv.py -q -m gpu --timeout 300 --timeout-method thread -rf > $OUT/${TAG}_tests.log 2>&1
RC=$?; echo "tests rc=$RC"; grep -E "passed|failed|FAIL|Error" $OUT/${TAG}_tests.log | tail -8
[ $RC -le 1 ] || exit $RC
timeout -k 10 300 python bench.py > $OUT/${TAG}_bench.log 2>&1 || { echo "bench failed"; tail -5 $OUT/${TAG}_bench.log; exit 1; }
tail -1 $OUT/${TAG}_bench.log | cut -c1-900
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/${TAG}_prof.log 2>&1 || { echo "prof failed"; exit 1; }
python $GRAFT_REPO_ROOT/tools/prof_summary.py $OUT/${TAG}_prof 7 > $OUT/${TAG}_kernel_stats.md
head -16 $OUT/${TAG}_kernel_stats.md | cut -c1-200
