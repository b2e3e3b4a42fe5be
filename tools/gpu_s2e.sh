#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_spectral.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s2e_tests.log 2>&1; rc=$?
tail -2 gpurun_out/s2e_tests.log; [ $rc -eq 0 ] || exit 1
for W in clkd; do
  echo "$W:"; SEL_LIB=dl-speech-enhancement_amd/sel/libsel_$W.so timeout -k 10 120 python tools/stft_clock.py 2>&1 | grep -v amdgpu.ids | tail -22 || exit 1
done
bash tools/gpu_s2c.sh s2e vmar0 dyn2
