#!/bin/bash
# conv_bench A/B of two libraries on the C3 shapes: tools/cb_ab.sh <lib_a> <lib_b> [shape filter]
cd $GRAFT_REPO_ROOT
for lib in "$1" "$2"; do
  echo "== $lib"
  SEL_LIB=$PWD/$lib SHAPE="$3" timeout -k 10 300 python tools/conv_bench.py 30 || exit 1
done
