#!/bin/bash
# A/B of kernel-selection knobs on the full bench: tools/ab_tune.sh "cfg1" "cfg2" ...
# (each cfg is a SEL_TUNE string, e.g. "4=1" or "7=1,6=4", optionally followed
# by "|VAR=val|..." environment settings; "" = defaults; run
# the list twice for an alternating A/B).  BENCH_ARGS: extra bench.py arguments
# (e.g. "--config c5 --steps 10 --warmup 2"; default: C3, 30 steps).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
ARGS=${BENCH_ARGS:---steps 30 --warmup 5}
i=0
for cfg in "$@"; do
  i=$((i + 1))
  tune=${cfg%%|*}
  envs=""
  [[ "$cfg" == *"|"* ]] && envs=${cfg#*|} && envs=${envs//|/ }
  tag=${cfg//[,|=\/]/_}; tag=${tag:0:60}
  env SEL_TUNE=$tune $envs timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline --no-fp32-companion > gpurun_out/ab_${i}_$tag.log 2>&1 || exit 1
  echo "cfg=$cfg $(tail -1 gpurun_out/ab_${i}_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("mean", d["ms_per_step"], "median", d["median_ms_per_step"], d["value"], d["roofline"]["kernel"], d["roofline"]["frac"])')"
done
