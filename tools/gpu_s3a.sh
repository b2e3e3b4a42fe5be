#!/bin/bash
# Discriminator layers on the warp-specialised kernel: parity tests, then C5 A/B
# (tune key 21: 0 = ws tiles, 1 = k_dconv_pf), alternating.  usage: tools/gpu_s3a.sh TAG
set -o pipefail
TAG=${1:-s3a}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -rf > $OUT/${TAG}_tests.log 2>&1
RC=$?; echo "tests rc=$RC"; tail -3 $OUT/${TAG}_tests.log
[ $RC -eq 0 ] || exit 1
for cfg in ${CFGS:-21=1 0=0 21=1 0=0}; do
  tag=x${cfg//=/_}
  SEL_TUNE=$cfg timeout -k 10 200 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/${TAG}_c5_$tag.log 2>&1 || exit 1
  echo "cfg=$cfg $(tail -1 $OUT/${TAG}_c5_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_ms_per_step"], d["value"])')"
done
