#!/bin/bash
# queue a gpurun call: retry only while no GPU slot is free (exit 3: nothing ran, nothing charged)
out=$1; shift
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun "$@" > "$out" 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 90
done
exit 3
