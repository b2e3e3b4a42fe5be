#!/bin/bash
# A/B of kernel-selection knobs on the full C3 bench: tools/ab_tune.sh "cfg1" "cfg2" ...
# (each cfg is a SEL_TUNE string, e.g. "4=1" or "7=1,6=4"; "" = defaults)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for cfg in "$@"; do
  tag=${cfg//,/_}
  SEL_TUNE=$cfg timeout -k 10 150 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab_$tag.log 2>&1 || exit 1
  echo "cfg=$cfg $(tail -1 gpurun_out/ab_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
