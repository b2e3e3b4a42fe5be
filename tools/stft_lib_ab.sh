#!/bin/bash
# STFT |X| probe (bench.py's stft_kernel line) under alternative libsel builds:
# tools/stft_lib_ab.sh libsel_a.so ...  ("" = the default), three alternating rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for pass in 1 2 3; do
  for L in "" "$@"; do
    if [ -n "$L" ]; then export SEL_LIB=dl-speech-enhancement_amd/sel/$L; else unset SEL_LIB; fi
    timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fp32-companion \
      > gpurun_out/stftab_${L:-default}.log 2>&1 || exit 1
    echo "${L:-default}: $(tail -1 gpurun_out/stftab_${L:-default}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read())["stft_kernel"]; print(d["median_launch_us"], d["frac_of_copy_f4"], d["copy_f4_GBs"])')"
  done
done
