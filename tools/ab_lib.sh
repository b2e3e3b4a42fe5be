#!/bin/bash
# RU kernel timings (tools/ru_bench.py, 32 and 64 channels) and the full C3 step
# for alternative builds of libsel: tools/ab_lib.sh libsel_a.so libsel_b.so ...
# ("" = the default libsel.so); each list is run twice, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
for pass in 1 2; do
  for L in "" "$@"; do
    if [ -n "$L" ]; then export SEL_LIB=dl-speech-enhancement_amd/sel/$L; else unset SEL_LIB; fi
    for C in 32 64; do
      RU_C=$C timeout -k 10 120 python tools/ru_bench.py > gpurun_out/abl_${L:-default}_$C.log 2>&1 || exit 1
      echo "${L:-default} C=$C: $(grep -E 'dil 9' gpurun_out/abl_${L:-default}_$C.log | cut -c1-200)"
    done
  done
done
unset SEL_LIB
CFGS=("")
for L in "$@"; do CFGS+=("|SEL_LIB=dl-speech-enhancement_amd/sel/$L"); done
bash tools/ab_tune.sh "${CFGS[@]}" "${CFGS[@]}"
