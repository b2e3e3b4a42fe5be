#!/bin/bash
# Full GPU tests, then C3 A/B of env settings (alternating).  usage: ENVS="A=1 B=2" tools/gpu_s3d.sh TAG
set -o pipefail
TAG=${1:-s3d}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -rf > $OUT/${TAG}_tests.log 2>&1
RC=$?; echo "tests rc=$RC"; tail -3 $OUT/${TAG}_tests.log
[ $RC -eq 0 ] || exit 1
for e in ${ENVS:-X=0}; do
  env $e timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-companion > $OUT/${TAG}_c3_$e.log 2>&1 || exit 1
  echo "$e $(tail -1 $OUT/${TAG}_c3_$e.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_ms_per_step"], d["value"], d["roofline"]["kernel"], d["roofline"]["frac"])')"
done
