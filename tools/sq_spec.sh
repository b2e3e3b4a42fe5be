#!/bin/bash
# stft |X| fwd timing + LDS counters per libsel variant: tools/sq_spec.sh p3 p4 ...
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for V in "$@"; do
  echo "== $V"
  SEL_LIB=dl-speech-enhancement_amd/sel/libsel_$V.so timeout -k 10 120 python tools/stft_bench.py 512 > gpurun_out/sb_$V.log 2>&1 || exit 1
  grep "stft_mag_fwd\|stft_loss_fwd\|mel loss" gpurun_out/sb_$V.log
  (cd /tmp && export TMPDIR=/tmp && SEL_LIB=$GRAFT_REPO_ROOT/dl-speech-enhancement_amd/sel/libsel_$V.so timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVES --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/sq_$V -o run -- python $GRAFT_REPO_ROOT/tools/stft_one.py > /dev/null 2>&1) || exit 1
  python tools/pmc_sq.py $(find gpurun_out/sq_$V -name "*counter_collection.csv") | grep stft_mag
done
