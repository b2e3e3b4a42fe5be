#!/bin/bash
# GPU session: conv microbench A/B, parity tests, smoke, bench, rocprof kernel stats.
# Usage: tools/gpu_round2.sh <tag> [pytest selection]
set -o pipefail
TAG=${1:-run}; shift
TESTS=${@:-tests}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 240 python -u tools/conv_bench.py 30 0 > $OUT/${TAG}_convbench.md 2>&1
RC=$?; echo "convbench rc=$RC"; cat $OUT/${TAG}_convbench.md | tail -20
[ $RC -eq 0 ] || exit $RC
timeout -k 10 600 python -u -m pytest $TESTS -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
RC=$?; echo "tests rc=$RC"; tail -5 $OUT/${TAG}_tests.log
[ $RC -le 1 ] || exit $RC
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1 || exit 1
tail -1 $OUT/${TAG}_smoke.log
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/${TAG}_bench.log 2>&1 || exit 1
tail -1 $OUT/${TAG}_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/${TAG}_prof.log 2>&1
echo "prof rc=$?"
