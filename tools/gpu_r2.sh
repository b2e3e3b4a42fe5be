#!/bin/bash
# GPU session: all -m gpu tests (no -x: report every failure), smoke, bench.
# Usage: tools/gpu_r2.sh <tag> [pytest selection...]
set -o pipefail
TAG=${1:-run}; shift
SEL=${@:-tests}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest $SEL -q -m gpu --timeout 150 --timeout-method thread -rf > $OUT/${TAG}_tests.log 2>&1
RC=$?; echo "tests rc=$RC"; tail -25 $OUT/${TAG}_tests.log
[ $RC -le 1 ] || exit $RC
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1 || exit 1
tail -1 $OUT/${TAG}_smoke.log
timeout -k 10 400 python bench.py > $OUT/${TAG}_bench.log 2>&1 || exit 1
tail -1 $OUT/${TAG}_bench.log
