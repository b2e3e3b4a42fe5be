#!/bin/bash
# fused RU kernels (tools/ru_bench.py) for alternative libsel builds, alternating:
#   tools/ab_ru.sh C libsel_a.so libsel_b.so ...   ("" = the default libsel.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
C=$1
shift
for pass in 1 2; do
  for L in "$@"; do
    if [ -n "$L" ]; then export SEL_LIB=dl-speech-enhancement_amd/sel/$L; else unset SEL_LIB; fi
    RU_C=$C timeout -k 10 120 python tools/ru_bench.py > gpurun_out/abru_${L:-default}_$C.log 2>&1 || exit 1
    echo "${L:-default} C=$C:"; grep -E '^dil' gpurun_out/abru_${L:-default}_$C.log | cut -c1-140
  done
done
