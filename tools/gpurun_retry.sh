#!/bin/bash
# gpurun with a bounded wait for a free box: retries ONLY when gpurun reports
# that no box / slot is free (exit 3, nothing ran, nothing charged), at most 6
# times, 90 s apart.  usage: tools/gpurun_retry.sh TIMEOUT 'command'
T=$1; shift
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout $T -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[retry] no box free (attempt $i), waiting 90 s" >&2
  sleep 90
done
exit 3
