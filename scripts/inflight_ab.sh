#!/bin/bash
# A/B of the in-flight cap and AQL queue count at host-bound sizes (native node ladder), one box.
# Output: gpurun_out/inflight_ab.jsonl
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "8 4" "12 4" "16 4" "12 8" "16 8"; do
    set -- $cfg
    DORA_GPU_MAX_IN_FLIGHT=$1 DORA_GPU_AQL_QUEUES=$2 timeout -k 10 120 python scripts/native_tp.py \
      --sizes "${SIZES:-1048576,4096000}" --n 5000 \
      | sed "s/^{/{\"in_flight\": $1, \"aql_queues\": $2, /" >> gpurun_out/inflight_ab.jsonl || exit $?
  done
done
