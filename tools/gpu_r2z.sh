#!/bin/bash
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-r2z}
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_gan.py -q -m gpu --timeout 200 --timeout-method thread -rf > $OUT/${TAG}_tests.log 2>&1
RC=$?; echo "tests rc=$RC"; grep -E "passed|failed|FAIL|Error" $OUT/${TAG}_tests.log | tail -8
[ $RC -le 1 ] || exit $RC
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-fp32-companion > $OUT/${TAG}_prof.log 2>&1
echo "prof rc=$?"; tail -1 $OUT/${TAG}_prof.log | cut -c1-300
python $GRAFT_REPO_ROOT/tools/prof_summary.py $OUT/${TAG}_prof 4 > $OUT/${TAG}_c5_kernel_stats.md
head -16 $OUT/${TAG}_c5_kernel_stats.md | cut -c1-180
