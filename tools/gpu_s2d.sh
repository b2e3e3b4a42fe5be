#!/bin/bash
# effective clock per ablation variant + FFT-only timing
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for W in clk8; do
  echo "$W:"; SEL_LIB=dl-speech-enhancement_amd/sel/libsel_$W.so timeout -k 10 120 python tools/stft_clock.py 2>&1 | tail -16 || exit 1
done
for W in; do
  SEL_LIB=dl-speech-enhancement_amd/sel/libsel_$W.so timeout -k 10 120 python tools/stft_bench.py 512 > gpurun_out/s2d_sb_$W.log 2>&1 || exit 1
  echo "$W: $(grep 'stft_mag_fwd | 1024' gpurun_out/s2d_sb_$W.log)"
done
