#!/bin/bash
# kernel-trace durations of the conv variants (no CPU-side timing)
OUT=$GRAFT_REPO_ROOT/gpurun_out
TAG=${1:-r2m}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof -o run -- \
  python $GRAFT_REPO_ROOT/tools/ws_probe.py "RU256 k7d1 fwd,RU256 k7 dgrad,down2 640->256 k3" ${2:-0,4} 27,24 > $OUT/${TAG}.log 2>&1 || { echo "prof failed"; tail -5 $OUT/${TAG}.log; exit 1; }
python $GRAFT_REPO_ROOT/tools/prof_summary.py $OUT/${TAG}_prof 1 > $OUT/${TAG}_stats.md
grep -E "k_conv" $OUT/${TAG}_stats.md | cut -c1-220
