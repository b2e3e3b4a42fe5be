#!/bin/bash
# PMC traffic for the C3 bench: two separate rocprofv3 passes (FETCH_SIZE, WRITE_SIZE),
# counters only (no sys/runtime trace), then per-kernel bytes/launch.  Usage: tools/pmc_round.sh <tag>
set -o pipefail
TAG=${1:-pmc}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C --output-format csv -d $OUT/${TAG}_$C -o run -- \
    python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fp32-companion > $OUT/${TAG}_$C.log 2>&1 || exit 1
  echo "$C done"
done
F=$(find $OUT/${TAG}_FETCH_SIZE -name "*counter_collection.csv" | head -1)
W=$(find $OUT/${TAG}_WRITE_SIZE -name "*counter_collection.csv" | head -1)
python $GRAFT_REPO_ROOT/tools/pmc_traffic.py "$F" "$W" $OUT/${TAG}_traffic.json 4 > $OUT/${TAG}_traffic.md
rm -f "$F" "$W"
head -16 $OUT/${TAG}_traffic.md
