#!/bin/bash
# Spectral A/B: parity tests + stft_bench for each libsel variant given (W2 W3 W4 ...)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for W in "$@"; do
  echo "== $W"
  SEL_LIB=dl-speech-enhancement_amd/sel/libsel_$W.so timeout -k 10 300 python -u -m pytest tests/test_gpu_spectral.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/spec_$W.log 2>&1; tail -2 gpurun_out/spec_$W.log
  SEL_LIB=dl-speech-enhancement_amd/sel/libsel_$W.so timeout -k 10 120 python tools/stft_bench.py 512 > gpurun_out/sbench_$W.log 2>&1 || exit 1
  grep "|" gpurun_out/sbench_$W.log | tail -8; grep copy gpurun_out/sbench_$W.log
done
