#!/bin/bash
# Deeper pipelines for host-bound sizes: in-flight cap (12 default below 8 MiB) x AQL queues,
# native node ladder at 1 MB / 4 MB, 5000 messages.  Output: gpurun_out/inflight_deep_ab.jsonl
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "12 4" "16 4" "24 4" "32 4" "24 8" "12 4" "24 4"; do
  set -- $spec
  timeout -k 10 150 python scripts/native_tp.py --sizes 1048576,4194304 --n 5000 \
    --env DORA_GPU_MAX_IN_FLIGHT=$1 --env DORA_GPU_AQL_QUEUES=$2 \
    >> gpurun_out/inflight_deep_ab.jsonl || exit $?
done
