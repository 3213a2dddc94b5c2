#!/bin/bash
# A/B of the headline pack's dispatch path on one box: 40.96 MB over the HIP fill streams
# (default) vs the AQL queues (DORA_GPU_AQL_MAX_BYTES above the sample), 20 and 1000 steps.
# Appends one JSON line per run to gpurun_out/headline_ab.jsonl.
export TMPDIR=/tmp
out=gpurun_out/headline_ab.jsonl
mkdir -p gpurun_out
run() {
  tag=$1; shift
  for steps in 20 1000; do
    line=$(env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --no-ladder --steps $steps --warmup 5) || exit $?
    echo "{\"tag\": \"$tag\", \"steps\": $steps, \"bench\": $line}" >> $out
  done
}
run hip DORA_GPU_AQL_MAX_BYTES=33554432
run aql4 DORA_GPU_AQL_MAX_BYTES=100000000 DORA_GPU_AQL_QUEUES=4
run aql3 DORA_GPU_AQL_MAX_BYTES=100000000 DORA_GPU_AQL_QUEUES=3
run aql2 DORA_GPU_AQL_MAX_BYTES=100000000 DORA_GPU_AQL_QUEUES=2
run hip DORA_GPU_AQL_MAX_BYTES=33554432
run aql3 DORA_GPU_AQL_MAX_BYTES=100000000 DORA_GPU_AQL_QUEUES=3
