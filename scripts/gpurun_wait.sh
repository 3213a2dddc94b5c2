#!/bin/bash
# Retry a gpurun call only while it reports no box/slot (exit 3: nothing ran, nothing charged).
# usage: gpurun_wait.sh <log> <timeout> <command>
log=$1; to=$2; cmd=$3
for i in $(seq 1 15); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 200
done
exit 3
