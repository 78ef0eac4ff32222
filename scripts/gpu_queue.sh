#!/bin/bash
# (builder tool) queue a gpurun call: retry only while no GPU slot is free (exit code 3)
log=$1; shift
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun "$@" > $log 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q -E "GPU slot\(s\) on this pod are busy|no free box right now" $log; then break; fi
  sleep 90
done
echo "RC=$rc" >> $log
