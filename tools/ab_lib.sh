cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py > gpurun_out/h_t.log 2>&1; tail -1 gpurun_out/h_t.log
for L in ${AB_ORDER:-prev new prev new}; do
  if [ $L = prev ]; then export SEL_LIB=$GRAFT_REPO_ROOT/dl-speech-enhancement_amd/sel/libsel_prev.so; else unset SEL_LIB; fi
  timeout -k 10 150 python bench.py --steps 30 --no-cpu-baseline > gpurun_out/ab_$L.log 2>&1 || exit 1
  echo "$L $(tail -1 gpurun_out/ab_$L.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
