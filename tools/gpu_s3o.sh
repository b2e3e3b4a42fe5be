#!/bin/bash
# GAN tests default and with SEL_TUNE=$ALT, then C5 A/B ($ALT vs default).  usage: ALT=28=1 tools/gpu_s3o.sh TAG
set -o pipefail
TAG=${1:-s3o}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_gan.py tests/test_gpu_dconv_variants.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/${TAG}_t0.log 2>&1 || { tail -3 $OUT/${TAG}_t0.log; exit 1; }
tail -1 $OUT/${TAG}_t0.log
SEL_TUNE=$ALT timeout -k 10 300 python -u -m pytest tests/test_gpu_gan.py tests/test_gpu_dconv_variants.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/${TAG}_t1.log 2>&1 || { tail -3 $OUT/${TAG}_t1.log; exit 1; }
tail -1 $OUT/${TAG}_t1.log
for cfg in $ALT 0=0 $ALT 0=0; do
  SEL_TUNE=$cfg timeout -k 10 200 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/${TAG}_c5_$cfg.log 2>&1 || exit 1
  echo "cfg=$cfg $(tail -1 $OUT/${TAG}_c5_$cfg.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_ms_per_step"], d["value"])')"
done
