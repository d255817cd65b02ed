#!/usr/bin/env bash
# gpurun with retries while no box is free (exit 3: nothing ran, nothing
# charged); any other exit -- success or a failing command -- ends it.
#   scripts/gpurun_retry.sh TIMEOUT 'COMMAND'
T=$1; shift
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 120
done
exit 3
