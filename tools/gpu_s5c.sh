#!/bin/bash
# spectral frame-kernel iteration sweep (tune key 14) under rocprof: per-kernel
# averages of the frame kernels for each setting.  usage: CFGS="14=0 14=1" tools/gpu_s5c.sh TAG
set -o pipefail
TAG=${1:-s5c}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for cfg in ${CFGS:-14=0 14=1 14=2 14=-1}; do
  SEL_TUNE=$cfg timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_$cfg -o run -- \
    python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fp32-companion > $OUT/${TAG}_$cfg.log 2>&1 || exit 1
  echo "== $cfg $(tail -1 $OUT/${TAG}_$cfg.log | cut -c1-120)"
  python - $OUT/${TAG}_$cfg <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "spec::" in r["Name"]:
        print(f"  {r['Name'][:60]:60s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:8.1f}")
PY
done
