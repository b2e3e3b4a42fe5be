#!/bin/bash
# C3 A/B of environment settings (alternating).  usage: ENVS="A=1 X=0" tools/gpu_s5f.sh TAG
set -o pipefail
TAG=${1:-s5f}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
i=0
for e in ${ENVS:-X=0}; do
  i=$((i+1))
  env $e timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-companion > $OUT/${TAG}_$i.log 2>&1 || exit 1
  echo "$e $(tail -1 $OUT/${TAG}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_ms_per_step"], d["value"])')"
done
