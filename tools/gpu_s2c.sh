#!/bin/bash
# stft_bench only, alternating the libsel variants given.  usage: gpu_s2c.sh TAG V1 V2 ...
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=$1; shift
for rep in 1 2; do
  for W in "$@"; do
    SEL_LIB=dl-speech-enhancement_amd/sel/libsel_$W.so timeout -k 10 120 python tools/stft_bench.py 512 > gpurun_out/${TAG}_sb_${W}_$rep.log 2>&1 || exit 1
    echo "$W rep $rep: $(grep 'stft_mag_fwd | 1024' gpurun_out/${TAG}_sb_${W}_$rep.log)"
  done
done
