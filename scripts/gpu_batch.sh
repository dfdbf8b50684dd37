#!/bin/bash
# Run several GPU steps in one gpurun call; each step has its own time limit.  A plain failure
# (pytest rc 1) moves on to the next step; a fault / abort / timeout (rc >= 124) stops the call.
# usage: bash scripts/gpu_batch.sh OUTDIR 'label|seconds|command' ...
O=$1; shift
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
for step in "$@"; do
  label=${step%%|*}; rest=${step#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "== $label ($secs s): $cmd"
  timeout -k 10 $secs bash -c "$cmd" > $O/$label.log 2>&1
  rc=$?
  echo "== $label rc=$rc"; tail -3 $O/$label.log
  if [ $rc -ge 124 ]; then echo "stopping after $label (rc=$rc)"; exit $rc; fi
done
