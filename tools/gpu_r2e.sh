#!/bin/bash
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_gan.py -q -m gpu --timeout 200 --timeout-method thread -rf > $OUT/r2e_tests.log 2>&1
RC=$?; echo "tests rc=$RC"; grep -E "passed|failed|FAIL" $OUT/r2e_tests.log | tail -8
[ $RC -le 1 ] || exit $RC
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r2e_prof -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/r2e_prof.log 2>&1
echo "prof rc=$?"; tail -1 $OUT/r2e_prof.log | cut -c1-400
python $GRAFT_REPO_ROOT/tools/prof_summary.py $OUT/r2e_prof 4 > $OUT/r2e_c5_kernel_stats.md
head -30 $OUT/r2e_c5_kernel_stats.md
