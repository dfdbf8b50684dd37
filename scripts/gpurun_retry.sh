#!/bin/bash
# gpurun with retries ONLY while no box / slot is free (exit 3: nothing ran, nothing charged).
# Any other outcome (success, failure, fault, timeout) is returned as is -- never re-run.
# usage: scripts/gpurun_retry.sh LOGFILE TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $LOG 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "no free box\|slot(s) on this pod are busy" $LOG; then exit $rc; fi
  echo "[retry $i: no box]" >> $LOG.retries
  sleep 60
done
exit 3
