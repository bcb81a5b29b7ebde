#!/bin/bash
# gpurun with retries while the pool has no free slot / box (exit 3: nothing ran, nothing charged).
# usage: tools/r4/gpurun_retry.sh TIMEOUT_S LOG 'command'
T=$1; LOG=$2; shift 2
for i in $(seq 1 ${RETRIES:-6}); do
  timeout $((T + 900)) /usr/local/graft/bin/gpurun --timeout $T -- "$@" > $LOG 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "attempt $i: no slot (rc 3), retrying" >> $LOG.retries
  sleep 90
done
exit 3
