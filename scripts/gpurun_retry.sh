#!/bin/bash
# Run a gpurun command; if the infrastructure reports a transient/back-off (nothing ran,
# nothing charged), wait and submit again (at most 6 times).  Any real run -- pass or fail --
# is never repeated.
for i in 1 2 3 4 5 6; do
  out=$(/usr/local/graft/bin/gpurun "$@" 2>&1)
  echo "$out" | tail -4
  if echo "$out" | grep -q "status=transient\|backing off\|no box\|slot free"; then
    sleep 45
    continue
  fi
  break
done
