# A/B of environment settings on the C3 bench (graph replay), alternating rounds:
#   AB_VARS="SEL_TUNE=59=0 SEL_TUNE=59=23" AB_ROUNDS=2 bash tools/ab_env.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
for i in $(seq ${AB_ROUNDS:-2}); do
  for v in $AB_VARS; do
    tag=$(echo "$v" | tr '=,/' '___')
    env $v timeout -k 10 200 python bench.py --no-cpu-baseline --no-fp32-companion --steps ${AB_STEPS:-30} > gpurun_out/ab_${tag}_$i.log 2>&1 || exit 1
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_${tag}_$i.log').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['median_ms_per_step'])"
  done
done
