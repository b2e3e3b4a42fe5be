#!/bin/bash
# Timing ablations of k_pw_bf16 (rocprof kernel stats, RU256 1x1 shapes): the
# default library and diagnostic builds with -DSEL_PW_ABL=1/2/4/8 linked as
# dl-speech-enhancement_amd/sel/libsel_abl<N>.so (conv.hip compiled with the
# define, linked with the other objects of csrc/build); run on the GPU box.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in "" 1 2 4 8; do
  lib=dl-speech-enhancement_amd/sel/libsel${v:+_abl$v}.so
  SEL_LIB=$PWD/$lib SHAPE='RU256 1x1' timeout -k 10 100 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pwabl$v -o run -- python tools/conv_bench.py 42 > gpurun_out/pwabl$v.log 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/pwabl$v/run_kernel_stats.csv')):
    if 'pw_bf16' in r['Name']: print('abl$v', r['Name'][:60], r['Calls'], r['AverageNs'])
"
done
