#!/bin/bash
# Run GPU pytest selections one after another on the box; stop at the first step that
# did not end with "tests passed/failed" (rc 0/1): a fault, abort or timeout ends the call.
# usage: tools/gpu_tests.sh OUTPREFIX 'pytest args' ['pytest args' ...]
out=$1; shift
mkdir -p gpurun_out
i=0
for sel in "$@"; do
  i=$((i+1))
  eval "timeout -k 10 600 python -u -m pytest $sel -x -q -s --timeout 400 --timeout-method thread" \
      > gpurun_out/${out}_$i.log 2>&1
  rc=$?
  echo "step $i rc $rc: $sel" | tee -a gpurun_out/${out}_steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
exit 0
