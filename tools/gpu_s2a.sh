#!/bin/bash
# STFT LDS-read A/B: parity tests on the default lib, alternating stft_bench runs
# of the variants given, SQ counter passes per variant.  usage: gpu_s2a.sh TAG V1 V2 ...
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 300 python -u -m pytest tests/test_gpu_spectral.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for W in "$@"; do
    SEL_LIB=dl-speech-enhancement_amd/sel/libsel_$W.so timeout -k 10 120 python tools/stft_bench.py 512 > gpurun_out/${TAG}_sb_${W}_$rep.log 2>&1 || exit 1
    echo "== $W rep $rep"; grep "|" gpurun_out/${TAG}_sb_${W}_$rep.log | tail -5
  done
done
cd /tmp && export TMPDIR=/tmp
for W in "$@"; do
  i=0
  for C in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"; do
    i=$((i+1))
    D=$GRAFT_REPO_ROOT/gpurun_out/${TAG}_sq_$W/p$i; mkdir -p $GRAFT_REPO_ROOT/gpurun_out/${TAG}_sq_$W
    SEL_LIB=$GRAFT_REPO_ROOT/dl-speech-enhancement_amd/sel/libsel_$W.so timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d $D -o run -- python $GRAFT_REPO_ROOT/tools/stft_one.py > $D.log 2>&1 || { echo "pass $i failed"; tail -3 $D.log; exit 1; }
  done
  echo "== SQ $W"
  python $GRAFT_REPO_ROOT/tools/pmc_sq.py $(find $GRAFT_REPO_ROOT/gpurun_out/${TAG}_sq_$W -name "*counter_collection.csv") | grep -i "stft_mag_fwd\|kernel" | tee $GRAFT_REPO_ROOT/gpurun_out/${TAG}_sq_$W.md
done
