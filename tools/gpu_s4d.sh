#!/bin/bash
# C5 A/B of environment settings (alternating).  usage: ENVS="A=1 X=0" tools/gpu_s4d.sh TAG
set -o pipefail
TAG=${1:-s4d}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for e in ${ENVS:-X=0}; do
  env $e timeout -k 10 200 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/${TAG}_c5_$e.log 2>&1 || exit 1
  echo "$e $(tail -1 $OUT/${TAG}_c5_$e.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_ms_per_step"], d["value"])')"
done
