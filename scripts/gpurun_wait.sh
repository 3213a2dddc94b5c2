#!/bin/bash
# Retry a gpurun call only while nothing ran and nothing was charged: no box or slot (exit 3), or
# the box taken away before the command started ("status=transient").
# usage: gpurun_wait.sh <log> <timeout> <command>
log=$1; to=$2; cmd=$3
for i in $(seq 1 15); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$log"; then exit $rc; fi
  sleep 120
done
exit 3
