#!/bin/bash
# spectral parity tests on the default lib, then stft_bench A/B of the variants given
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 300 python -u -m pytest tests/test_gpu_spectral.py tests/test_gpu_melspec.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for W in "$@"; do
    SEL_LIB=dl-speech-enhancement_amd/sel/libsel_$W.so timeout -k 10 120 python tools/stft_bench.py 512 > gpurun_out/${TAG}_sb_${W}_$rep.log 2>&1 || exit 1
    echo "== $W rep $rep $(grep -i copy gpurun_out/${TAG}_sb_${W}_$rep.log)"; grep "stft_mag_fwd\|stft_loss_fwd\|mel" gpurun_out/${TAG}_sb_${W}_$rep.log
  done
done
