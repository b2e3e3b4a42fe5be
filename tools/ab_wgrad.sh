#!/bin/bash
# weight-gradient kernels (tools/conv_bench.py WGRAD=1, default path) for
# alternative libsel builds, alternating: tools/ab_wgrad.sh libsel_a.so ...  ("" = default)
set -o pipefail
cd $GRAFT_REPO_ROOT
for pass in 1 2; do
  for L in "$@"; do
    if [ -n "$L" ]; then export SEL_LIB=dl-speech-enhancement_amd/sel/$L; else unset SEL_LIB; fi
    WGRAD=1 WG_B=0 timeout -k 10 200 python tools/conv_bench.py > gpurun_out/abwg_${L:-default}.log 2>&1 || exit 1
    echo "${L:-default}:"; grep "^| " gpurun_out/abwg_${L:-default}.log | grep -v "wgrad shape" | cut -c1-90
  done
done
