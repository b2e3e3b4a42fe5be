#!/bin/bash
# packed-FMA shortx: dconv/GAN tests, then C5 A/B against the previous library (SEL_LIB)
set -o pipefail
TAG=${1:-s5h}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_dconv_variants.py tests/test_gpu_gan.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
RC=$?; echo "tests rc=$RC"; tail -2 $OUT/${TAG}_tests.log
[ $RC -eq 0 ] || exit 1
P=dl-speech-enhancement_amd/sel/libsel_prev.so
i=0
for e in SEL_LIB=$P X=0 SEL_LIB=$P X=0; do
  i=$((i+1))
  env $e timeout -k 10 200 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/${TAG}_c5_$i.log 2>&1 || exit 1
  echo "$e $(tail -1 $OUT/${TAG}_c5_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_ms_per_step"])')"
done
