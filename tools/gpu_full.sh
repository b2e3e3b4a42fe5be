#!/bin/bash
# Round-end style GPU session: parity tests, smoke, bench (with CPU baseline),
# rocprofv3 kernel stats of the bench.  Usage: tools/gpu_full.sh <tag>
set -o pipefail
TAG=${1:-run}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
RC=$?; echo "tests rc=$RC"; tail -2 $OUT/${TAG}_tests.log
[ $RC -le 1 ] || exit $RC
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1 || exit 1
tail -1 $OUT/${TAG}_smoke.log
timeout -k 10 400 python bench.py > $OUT/${TAG}_bench.log 2>&1 || exit 1
tail -1 $OUT/${TAG}_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/${TAG}_prof.log 2>&1
echo "prof rc=$?"
