#!/bin/bash
# Run one gpurun command, waiting for a free GPU slot: gpurun exits 3 when no
# box/slot is free (nothing ran, nothing charged); only that case is retried,
# every 3 minutes, at most 10 times.  Any other exit (including GPU failures)
# is returned as is.  Usage: tools/gpurun_when_free.sh <timeout_s> <command>
to=$1; shift
for i in $(seq 1 10); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[gpurun_when_free] no free slot (try $i), waiting 180 s"
  sleep 180
done
exit 3
