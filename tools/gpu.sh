#!/bin/bash
# One parameterised GPU-box runner (run through gpurun from the repo root).
#   tools/gpu.sh tests TAG [pytest args...]   pytest -m gpu (default: the whole GPU suite)
#   tools/gpu.sh bench TAG [bench args...]    bench.py -> gpurun_out/TAG_bench.log
#   tools/gpu.sh prof  TAG [bench args...]    rocprofv3 --kernel-trace --stats of bench.py -> TAG_kernel_stats.md
#   tools/gpu.sh pmc   TAG [bench args...]    FETCH_SIZE / WRITE_SIZE passes of bench.py -> TAG_traffic.{json,md}
#   tools/gpu.sh smoke TAG                    __graft_entry__.smoke()
# Every GPU step runs under its own timeout; the first failure ends the script.
set -o pipefail
CMD=$1
TAG=$2
shift 2
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out
mkdir -p $OUT
case $CMD in
  tests)
    ARGS=("$@")
    [ ${#ARGS[@]} -eq 0 ] && ARGS=(tests)
    cd $R && timeout -k 10 ${GPU_TIMEOUT:-900} python -u -m pytest -x -v -m gpu --timeout ${TEST_TIMEOUT:-300} \
      --timeout-method thread "${ARGS[@]}" > $OUT/${TAG}_tests.log 2>&1
    RC=$?; echo "tests rc=$RC"; grep -E "passed|failed|error" $OUT/${TAG}_tests.log | tail -3
    exit $RC ;;
  bench)
    cd $R && timeout -k 10 ${GPU_TIMEOUT:-600} python bench.py "$@" > $OUT/${TAG}_bench.log 2>&1
    RC=$?; tail -1 $OUT/${TAG}_bench.log | cut -c1-1500; exit $RC ;;
  prof)
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 ${GPU_TIMEOUT:-400} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof -o run -- \
      python $R/bench.py --no-cpu-baseline --no-fp32-companion "$@" > $OUT/${TAG}_prof.log 2>&1 || { echo "prof failed"; tail -5 $OUT/${TAG}_prof.log; exit 1; }
    python $R/tools/prof_summary.py $OUT/${TAG}_prof ${STEPS_PROF:-auto} > $OUT/${TAG}_kernel_stats.md
    tail -1 $OUT/${TAG}_prof.log | cut -c1-600
    head -25 $OUT/${TAG}_kernel_stats.md | cut -c1-220 ;;
  pmc)
    cd /tmp && export TMPDIR=/tmp
    for C in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 ${GPU_TIMEOUT:-400} rocprofv3 --pmc $C --output-format csv -d $OUT/${TAG}_$C -o run -- \
        python $R/bench.py --no-cpu-baseline --no-fp32-companion "$@" > $OUT/${TAG}_$C.log 2>&1 || { echo "$C failed"; exit 1; }
      echo "$C done"
    done
    F=$(find $OUT/${TAG}_FETCH_SIZE -name "*counter_collection.csv" | head -1)
    W=$(find $OUT/${TAG}_WRITE_SIZE -name "*counter_collection.csv" | head -1)
    python $R/tools/pmc_traffic.py "$F" "$W" $OUT/${TAG}_traffic.json ${STEPS_PMC:-auto} > $OUT/${TAG}_traffic.md
    rm -f "$F" "$W"
    head -16 $OUT/${TAG}_traffic.md ;;
  smoke)
    cd $R && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1
    RC=$?; tail -2 $OUT/${TAG}_smoke.log; exit $RC ;;
  *) echo "unknown command $CMD"; exit 2 ;;
esac
