#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first fatal exit
# (timeout, abort, segfault, signal).  Ordinary failures (e.g. a failing test) continue.
#   scripts/run_steps.sh "name:timeout_s:command" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; to=${rest%%:*}; cmd=${rest#*:}
  start=$(date +%s)
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc $(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
  if [ $rc -ge 124 ]; then echo "fatal exit $rc in $name; stopping"; exit $rc; fi
done
