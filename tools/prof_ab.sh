#!/bin/bash
# rocprofv3 kernel stats of the C3 bench under two environments: tools/prof_ab.sh "ENV_A" "ENV_B"
set -o pipefail
cd /tmp && export TMPDIR=/tmp
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pab_$i -o run -- \
    python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pab_$i.log 2>&1 || exit 1
  echo "== $E"; python $GRAFT_REPO_ROOT/tools/prof_summary.py $GRAFT_REPO_ROOT/gpurun_out/pab_$i 7 | head -16
done
