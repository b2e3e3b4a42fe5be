#!/bin/bash
# C3 A/B of SEL_TUNE settings (alternating), no tests.  usage: CFGS="a=1 0=0" tools/gpu_s3l.sh TAG
set -o pipefail
TAG=${1:-s3l}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for cfg in ${CFGS:-0=0}; do
  SEL_TUNE=$cfg timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-companion > $OUT/${TAG}_$cfg.log 2>&1 || exit 1
  echo "$cfg $(tail -1 $OUT/${TAG}_$cfg.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_ms_per_step"], d["value"])')"
done
